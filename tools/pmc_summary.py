#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc CSV (counter_collection.csv) per kernel: waves, MFMA utilisation
and the issue / wait shares of the wave cycles, averaged over dispatches.

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the busy
counter sums the matrix-pipe cycles of every SIMD (profiles/pmc_conv_r2.md).

  python tools/pmc_summary.py gpurun_out/pmc_x/.../run_counter_collection.csv
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    per = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> value
    for d in csv.DictReader(open(path)):
        name = re.sub(r"\(.*$", "", d.get("Kernel_Name", d.get("Kernel-Name", "?")))[:70]
        disp = d.get("Dispatch_Id", d.get("Dispatch-Id", "0"))
        per[(name, disp)][d.get("Counter_Name", d.get("Counter-Name"))] += float(d.get("Counter_Value", d.get("Counter-Value", 0)))
    agg = defaultdict(lambda: defaultdict(list))
    for (name, _), cs in per.items():
        for k, v in cs.items():
            agg[name][k].append(v)
    print("| kernel | dispatches | waves | MFMA util | active issue | waiting |")
    print("|---|---:|---:|---:|---:|---:|")
    for name, cs in sorted(agg.items()):
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        n = len(next(iter(cs.values())))
        gui = m.get("GRBM_GUI_ACTIVE", 0.0)
        util = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 1024) if gui else 0.0
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        act = m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else 0.0
        wait = m.get("SQ_WAIT_ANY", 0.0) / wc if wc else 0.0
        print(f"| `{name}` | {n} | {m.get('SQ_WAVES', 0):.0f} | {100 * util:.1f}% | {100 * act:.0f}% | {100 * wait:.0f}% |")


if __name__ == "__main__":
    main()
