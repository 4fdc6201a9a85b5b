#!/usr/bin/env python3
"""Which hipGraph captures of in-tree RCCL point-to-point calls survive `capture_end`?

Round 4 saw a segfault in `torch.cuda.graph.__exit__` (hipStreamEndCapture) on a graph holding
grouped rank-to-self send/recv on the RcclP2P communicators (one communicator + one forked side
stream per direction). Each variant below runs in its own subprocess (a crash ends only it) and
prints one JSON line: variant, env, exit code, and whether the replayed data was right.

  python tools/rccl_capture_probe.py            # all variants (needs a GPU)
  python tools/rccl_capture_probe.py --one V     # a single variant in this process
"""
import json
import os
import subprocess
import sys

VARIANTS = {
    # name: (communicators, side streams, captured, extra env); ordered from the expected-safe to
    # the variants that hung / crashed (the run stops at the first timeout)
    "eager_1comm": (1, False, False, {}),
    "cap_allreduce_2comm_side": (2, True, True, {"_COLL": "1"}),
    # ProcessGroupNCCL (c10d) at world 1: reduce_scatter_tensor + all_gather_into_tensor, async +
    # wait, captured on the capture stream itself or on a forked side stream
    "c10d_rsag_eager": (1, False, False, {"_C10D": "1"}),
    "c10d_allreduce_side": (1, True, True, {"_C10D": "1", "_COLL": "1"}),
    "c10d_rsag_capstream": (1, False, True, {"_C10D": "1"}),
    "c10d_rsag_side": (1, True, True, {"_C10D": "1"}),
    "cap_1comm_side": (1, True, True, {}),
    "cap_2comm_side": (2, True, True, {}),
    "cap_2comm_side_nomix": (2, True, True, {"NCCL_GRAPH_MIXING_SUPPORT": "0"}),
    "cap_1comm_capstream_nomix": (1, False, True, {"NCCL_GRAPH_MIXING_SUPPORT": "0"}),
    "cap_1comm_capstream": (1, False, True, {}),
}


def run_one(name):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    from dcnn_amd.ops._ext import kernels
    from dcnn_amd.parallel.rccl import RcclCommunicator
    ncomm, side, captured, env = VARIANTS[name]
    coll = env.get("_COLL") == "1"
    c10d = env.get("_C10D") == "1"
    K = kernels()
    if c10d:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("PROBE_PORT", "29611"))
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))

        class _C10dComm:
            def all_reduce(self, t):
                dist.all_reduce(t, async_op=True).wait()

            def close(self):
                pass

        comms = [_C10dComm() for _ in range(ncomm)]
    else:
        comms = [RcclCommunicator(0, 1, torch.device("cuda", 0)) for _ in range(ncomm)]
    streams = [torch.cuda.Stream() for _ in range(ncomm)]
    src = [torch.randn(4096, device="cuda") for _ in range(ncomm)]
    dst = [torch.zeros_like(t) for t in src]

    def body():
        for c, s, a, b in zip(comms, streams, src, dst):
            ctx = torch.cuda.stream(s) if side else torch.cuda.stream(torch.cuda.current_stream())
            if side:
                s.wait_stream(torch.cuda.current_stream())
            with ctx:
                if coll:
                    b.copy_(a)
                    c.all_reduce(b)
                elif c10d:
                    import torch.distributed as dist
                    mid = torch.empty_like(a)
                    dist.reduce_scatter_tensor(mid, a, async_op=True).wait()
                    dist.all_gather_into_tensor(b, mid, async_op=True).wait()
                else:
                    K.rccl.group_start()
                    c.send(a, 0)
                    c.recv(b, 0)
                    K.rccl.group_end()
            if side:
                torch.cuda.current_stream().wait_stream(s)

    if captured:
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            with torch.cuda.graph(g, stream=cs):
                body()
        torch.cuda.current_stream().wait_stream(cs)
        g.replay()
    else:
        body()
    torch.cuda.synchronize()
    ok = all(torch.equal(a, b) for a, b in zip(src, dst))
    for c in comms:
        c.close()
    print(json.dumps({"variant": name, "ok": ok}), flush=True)
    return 0 if ok else 1


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        sys.exit(run_one(sys.argv[2]))
    for name, (_, _, _, env) in VARIANTS.items():
        e = dict(os.environ)
        e.update({k: v for k, v in env.items() if not k.startswith("_")})
        try:
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", name], env=e,
                               capture_output=True, text=True, timeout=60)
            rc, out = p.returncode, (p.stdout + p.stderr)
        except subprocess.TimeoutExpired:
            print(json.dumps({"variant": name, "rc": "timeout"}), flush=True)
            sys.exit(124)  # a hung GPU step: start nothing more on the GPU in this run
        ok = '"ok": true' in out
        print(json.dumps({"variant": name, "env": {k: v for k, v in env.items() if not k.startswith("_")},
                          "rc": rc, "ok": ok, "tail": out.strip().splitlines()[-3:] if out.strip() else []}),
              flush=True)


if __name__ == "__main__":
    main()
