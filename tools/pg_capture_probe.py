#!/usr/bin/env python3
"""Probe: ProcessGroupNCCL's watchdog vs hipGraph capture (world 1, one GPU).

Each round issues eager all-reduces, synchronises, then captures a graph that holds collectives
(thread-local capture mode, as runtime/step.py) and sleeps 0.25 s inside the capture, so a watchdog
pass (one every ~100 ms) always falls inside it. First hypothesis: the watchdog still lists the
eager works when the capture begins, and its query of their end events during the capture fails.
Result on the MI355X box (profiles/pg_capture_probe_r6.md): that hypothesis is FALSE (plain mode
survives 30 rounds); the abort comes from async_op=True collectives issued under capture (async
mode aborts in round 0): their works are listed for the watchdog although their end events were
recorded in the capture, and the watchdog's query of such an event fails with hipErrorCapturedEvent.

  python tools/pg_capture_probe.py --rounds 40 --mode plain|async|side|wire
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
    ap.add_argument("--eager", type=int, default=4, help="eager all-reduces before each capture")
    ap.add_argument("--mode", default="plain", choices=["plain", "async", "side", "wire"],
                    help="plain: blocking (async_op=False) all-reduces on the capture stream; async: "
                         "async_op=True works waited at the end of the capture (round 5's DataParallel torch "
                         "plane: aborts); side: blocking all-reduces issued from a comm stream forked from the "
                         "capture stream and joined back (the fixed plane); wire: blocking reduce_scatter_tensor "
                         "+ all_gather_into_tensor on a forked comm stream (the fixed bf16 wire)")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    x = torch.ones(1 << 20, device="cuda")
    s = torch.cuda.Stream()
    comm = torch.cuda.Stream()
    xb = torch.ones(1 << 16, device="cuda", dtype=torch.bfloat16)
    red = torch.empty(1 << 16, device="cuda", dtype=torch.bfloat16)
    graphs = []
    t0 = time.time()
    for r in range(a.rounds):
        for _ in range(a.eager):
            dist.all_reduce(x, async_op=True).wait()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            works = []
            for _ in range(8):
                if a.mode == "plain":
                    dist.all_reduce(x)
                elif a.mode == "async":
                    works.append(dist.all_reduce(x, async_op=True))
                elif a.mode == "side":
                    comm.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(comm):
                        dist.all_reduce(x)
                else:
                    comm.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(comm):
                        dist.reduce_scatter_tensor(red, xb)
                        dist.all_gather_into_tensor(xb, red)
                x.mul_(0.5)
            for w in works:
                w.wait()
            if a.mode in ("side", "wire"):
                torch.cuda.current_stream().wait_stream(comm)
            time.sleep(0.25)  # (host) a capture window that a watchdog pass (every ~100 ms) falls inside
        g.replay()
        torch.cuda.synchronize()
        graphs.append(g)
        print(f"round {r} ok ({time.time() - t0:.1f} s)", flush=True)
    print("PROBE OK", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
