#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite ``*_results.db`` or ``*_kernel_stats.csv``)
into a markdown table suitable for ``profiles/``.

Per-step times are normalised by the number of optimizer-kernel dispatches (one per
training step). From a rocpd database only the LAST steps are counted (``--last N``, default: all
but the first four steps): the window runs from the end of one optimizer dispatch to the end of
the N-th after it, so it holds graph replays only, not the eager warm-up steps, the capture's
warm-up or its allocator copies.

  python tools/prof_summary.py gpurun_out/prof6/run_results.db [--last 10] > profiles/resnet18_b256.md
"""
import csv
import os
import re
import sqlite3
import sys
from collections import defaultdict


def _short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*\)$", "", name)
    return name[:90]


def load(path, last=None):
    rows = defaultdict(lambda: [0, 0.0])
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        ks = list(c.execute("select name, start, end, duration from kernels order by start"))
        opt = [e for (n, _, e, _) in ks if "adam_kernel" in n or "sgd_kernel" in n]
        lo, hi = None, None
        if len(opt) >= 2:
            m = last if last else max(1, len(opt) - 4)
            m = min(m, len(opt) - 1)
            lo, hi = opt[-m - 1], opt[-1]  # after the (m+1)-th last optimizer dispatch .. the last one
        for name, st, en, dur in ks:
            if lo is not None and not (st > lo and en <= hi):
                continue
            r = rows[_short(name)]
            r[0] += 1
            r[1] += dur / 1e3  # ns -> us
    else:
        with open(path) as f:
            for d in csv.DictReader(f):
                r = rows[_short(d["Name"])]
                r[0] += int(d["Calls"])
                r[1] += float(d["TotalDurationNs"]) / 1e3
    return rows


def main():
    if len(sys.argv) < 2 or sys.argv[1].startswith("-") or not os.path.isfile(sys.argv[1]):
        sys.exit(__doc__)  # (sqlite3.connect would create an empty database at a bad path)
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else None
    rows = load(path, last)
    steps = sum(v[0] for k, v in rows.items() if "adam_kernel" in k or "sgd_kernel" in k) or 1
    total = sum(v[1] for v in rows.values())
    print(f"# Kernel summary: `{path}`\n")
    print(f"optimizer dispatches (= training steps in the replay window): {steps}; total GPU kernel time "
          f"{total / 1e3:.2f} ms; **{total / steps / 1e3:.3f} ms kernel time per step**\n")
    print("| kernel | calls | calls/step | total ms | us/step | % |")
    print("|---|---:|---:|---:|---:|---:|")
    for k, (n, us) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        if us / total < 0.002:
            continue
        print(f"| `{k}` | {n} | {n / steps:.1f} | {us / 1e3:.2f} | {us / steps:.1f} | {100 * us / total:.1f} |")


if __name__ == "__main__":
    main()
