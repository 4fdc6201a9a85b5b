#!/usr/bin/env python3
"""Probe: ProcessGroupNCCL's watchdog vs hipGraph capture (world 1, one GPU).

Each round issues eager all-reduces, synchronises, then captures a graph that holds an all-reduce
(thread-local capture mode, as runtime/step.py). Hypothesis under test: the watchdog thread
(one pass every ~100 ms) still lists the eager works when the capture begins; its query of their
end events while the PG's internal stream has been pulled into the capture fails
(hipErrorCapturedEvent / hipErrorStreamCaptureUnsupported) and the watchdog aborts the process.
With --drain the probe waits for the watchdog to retire the eager works first
(runtime/capture.py: drain_collective_watchdog).

  python tools/pg_capture_probe.py --rounds 40 [--drain]
Prints one line per round and "PROBE OK" at the end; an abort ends the process (SIGABRT).
"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--drain", action="store_true")
    ap.add_argument("--eager", type=int, default=4, help="eager all-reduces before each capture")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from dcnn_amd.runtime.capture import drain_collective_watchdog
    x = torch.ones(1 << 20, device="cuda")
    s = torch.cuda.Stream()
    graphs = []
    t0 = time.time()
    for r in range(a.rounds):
        for _ in range(a.eager):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        if a.drain:
            drain_collective_watchdog(force=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            for _ in range(8):
                dist.all_reduce(x)
                x.mul_(0.5)
            time.sleep(0.25)  # (host) a capture window that a watchdog pass (every ~100 ms) falls inside
        g.replay()
        torch.cuda.synchronize()
        graphs.append(g)
        print(f"round {r} ok ({time.time() - t0:.1f} s)", flush=True)
    print("PROBE OK", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
