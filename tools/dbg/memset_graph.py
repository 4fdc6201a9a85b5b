"""Debug: hipMemsetAsync (rt.memset_async) captured in a hipGraph, replayed; sizes / pools."""
import torch
from dcnn_amd.ops import hip
from dcnn_amd.device import get_gpu

for n in (1 << 10, 1 << 20, 11_300_000, 30_000_000):
    for src in ("torch", "native"):
        t = torch.ones(n, device="cuda") if src == "torch" else get_gpu(0).allocate(n, torch.float32)
        t.fill_(1.0)
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            hip.zero_(t)
        torch.cuda.synchronize()
        res = []
        for _ in range(2):
            t.fill_(1.0)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            res.append(float(t.abs().sum()))
        print(n, src, "after replays (expect 0):", res)
