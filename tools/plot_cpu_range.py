#!/usr/bin/env python3
"""Plot CPU utilisation over time for several processes (reference src/plot_cpu_range.py:1-118).

Reads the newest ``<prefix>_*.csv`` (columns ``t_sec, cpu_percent, tag``) for each prefix in
``--logs`` — the files ``dcnn_amd.utils.metrics.CpuUsageLogger`` writes, e.g. from pipeline
workers started with ``CPU_LOG_DIR=./logs`` — optionally clips to a time window and smooths with
a moving average, and saves one line per process to a PNG. ``--prefixes`` defaults to every
prefix found (the reference hard-codes coordinator / worker-8001 / worker-8002).

    python tools/plot_cpu_range.py --logs ./logs --out cpu_usage.png [--tmin 0 --tmax 5] [--smooth 3]
"""
import argparse
import csv
import glob
import os
import sys
from collections import deque


def newest_csv(logdir, prefix):
    files = glob.glob(os.path.join(logdir, f"{prefix}_*.csv"))
    if not files:
        raise FileNotFoundError(f"no CSV for prefix {prefix!r} in {logdir}")
    return max(files, key=os.path.getmtime)


def load_series(path):
    t, y, tag = [], [], None
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            t.append(float(row.get("t_sec", 0) or 0))
            y.append(float(row.get("cpu_percent", 0) or 0))
            tag = tag or row.get("tag")
    return tag or os.path.basename(path).split("_")[0], t, y


def moving_average(vals, k):
    if k <= 1:
        return list(vals)
    q, s, out = deque(), 0.0, []
    for v in vals:
        q.append(v)
        s += v
        if len(q) > k:
            s -= q.popleft()
        out.append(s / len(q))
    return out


def window(t, y, tmin, tmax):
    keep = [(a, b) for a, b in zip(t, y) if (tmin is None or a >= tmin) and (tmax is None or a <= tmax)]
    return [a for a, _ in keep], [b for _, b in keep]


def discover_prefixes(logdir):
    names = {os.path.basename(p).split("_")[0] for p in glob.glob(os.path.join(logdir, "*_*.csv"))}
    return sorted(names)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--logs", default="./logs")
    ap.add_argument("--out", default="cpu_usage.png")
    ap.add_argument("--prefixes", default="", help="comma list (default: all found)")
    ap.add_argument("--smooth", type=int, default=1)
    ap.add_argument("--tmin", type=float, default=None)
    ap.add_argument("--tmax", type=float, default=None)
    a = ap.parse_args(argv)
    prefixes = [p for p in a.prefixes.split(",") if p] or discover_prefixes(a.logs)
    if not prefixes:
        raise SystemExit(f"no CPU logs in {a.logs}")
    series = []
    for p in prefixes:
        path = newest_csv(a.logs, p)
        tag, t, y = load_series(path)
        t, y = window(t, y, a.tmin, a.tmax)
        if not t:
            print(f"[warning] series {tag!r} is empty in the requested window; skipped")
            continue
        series.append((tag, t, moving_average(y, a.smooth), path))
    if not series:
        raise SystemExit("nothing to plot (window too narrow?)")
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.figure(figsize=(18, 10))
    for tag, t, y, path in series:
        plt.plot(t, y, label=f"{tag}  (from: {os.path.basename(path)})")
    plt.xlabel("Time (s)")
    plt.ylabel("CPU Utilization (%)")
    title = "CPU usage per process"
    if a.tmin is not None or a.tmax is not None:
        title += f"  [window: {a.tmin if a.tmin is not None else '-'}-{a.tmax if a.tmax is not None else '-'} s]"
        lo = a.tmin if a.tmin is not None else min(s[1][0] for s in series)
        hi = a.tmax if a.tmax is not None else max(s[1][-1] for s in series)
        if lo < hi:
            plt.xlim(lo, hi)
    plt.title(title)
    plt.grid(True, alpha=0.3, linewidth=0.5)
    plt.legend()
    plt.tight_layout()
    plt.savefig(a.out, dpi=150)
    print(f"Saved: {a.out}")
    for s in series:
        print(" -", s[3])
    return 0


if __name__ == "__main__":
    sys.exit(main())
