#!/usr/bin/env python3
"""GPU occupancy of a traced run (rocprofv3 kernel trace, rocpd ``*_results.db``): over the last
N optimizer steps, the wall span, the union of kernel-busy intervals (any kernel running on any
stream), the idle time and its largest gaps, and how many kernels ran concurrently. Used to tell
a host/scheduling-bound run (idle gaps between kernels) from a device-bound one.

  python tools/gpu_busy.py gpurun_out/prof_x/run_results.db [more.db ...] [--steps 5] [--opt-per-step S]

(--opt-per-step: optimizer dispatches per training step, e.g. the stage count of a pipeline.
Several databases — one per process of a multi-process run on the same GPU, e.g. native pipeline
stage workers — are merged into one timeline: the device timestamps share one clock.)
"""
import sqlite3
import sys


def main():
    args, paths = sys.argv[1:], []
    while args and not args[0].startswith("--"):
        paths.append(args.pop(0))
    nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 5
    per = int(sys.argv[sys.argv.index("--opt-per-step") + 1]) if "--opt-per-step" in sys.argv else 1
    ks = []
    for path in paths:
        c = sqlite3.connect(path)
        ks += [(int(s), int(e), n) for s, e, n in c.execute("select start, end, name from kernels")]
    ks.sort()
    opt = [i for i, k in enumerate(ks) if "adam_kernel" in k[2] or "sgd_kernel" in k[2]][per - 1::per]
    if len(opt) < nsteps + 1:
        nsteps = max(1, len(opt) - 1)
    # window: from the end of the optimizer dispatch nsteps+1 from the end to the last one's end
    lo = ks[opt[-nsteps - 1]][1] if len(opt) > nsteps else ks[0][0]
    hi = ks[opt[-1]][1]
    win = [k for k in ks if k[1] > lo and k[0] < hi]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, _ in win:
        s, e = max(s, lo), min(e, hi)
        if cur_e is None:
            cur_s, cur_e = s, e
            if s > lo:
                gaps.append(s - lo)
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
        if hi > cur_e:
            gaps.append(hi - cur_e)
    span = hi - lo
    ksum = sum(min(e, hi) - max(s, lo) for s, e, _ in win)
    gaps.sort(reverse=True)
    print(f"steps {nsteps}: span {span / 1e6 / nsteps:.3f} ms/step, kernels {len(win) / nsteps:.0f}/step, "
          f"busy (union) {busy / 1e6 / nsteps:.3f} ms/step ({100 * busy / span:.1f}%), "
          f"idle {(span - busy) / 1e6 / nsteps:.3f} ms/step, summed kernel time {ksum / 1e6 / nsteps:.3f} ms/step "
          f"(mean concurrency while busy {ksum / max(busy, 1):.2f})")
    big = [g for g in gaps if g > 20_000]
    print(f"idle gaps > 20 us: {len(big) / nsteps:.1f}/step totalling {sum(big) / 1e6 / nsteps:.3f} ms/step; "
          f"largest {', '.join(f'{g / 1e3:.0f}' for g in gaps[:8])} us")


if __name__ == "__main__":
    main()
