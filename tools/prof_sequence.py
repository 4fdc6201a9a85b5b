#!/usr/bin/env python3
"""Print the kernel sequence of the LAST traced training step from a rocprofv3 rocpd database
(between the last two optimizer kernels), with gaps: shows where copies, fills and launch gaps
sit in a captured step.

  python tools/prof_sequence.py gpurun_out/prof_r2a/run_results.db [max_rows]
"""
import os
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*\)$", "", name)[:80]


def main():
    if len(sys.argv) < 2 or sys.argv[1].startswith("-") or not os.path.isfile(sys.argv[1]):
        sys.exit(__doc__)  # (sqlite3.connect would create an empty database at a bad path)
    path = sys.argv[1]
    limit = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    start = "start" if "start" in cols else "begin"
    rows = list(c.execute(f"select name, {start}, duration from kernels order by {start}"))
    opt = [i for i, r in enumerate(rows) if "adam_kernel" in r[0] or "sgd_kernel" in r[0]]
    if len(opt) < 2:
        sys.exit("need two optimizer dispatches in the trace")
    lo, hi = opt[-2] + 1, opt[-1] + 1
    t0 = rows[lo][1]
    prev_end = rows[lo - 1][1] + rows[lo - 1][2]
    busy = 0
    print(f"{'t_us':>9} {'gap_us':>7} {'dur_us':>7}  kernel")
    for name, st, dur in rows[lo:hi][:limit]:
        print(f"{(st - t0) / 1e3:9.1f} {(st - prev_end) / 1e3:7.1f} {dur / 1e3:7.1f}  {short(name)}")
        prev_end = st + dur
        busy += dur
    span = rows[hi - 1][1] + rows[hi - 1][2] - rows[lo][1]
    print(f"# {hi - lo} kernels, span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / span:.1f}%)")


if __name__ == "__main__":
    main()
