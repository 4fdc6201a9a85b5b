#!/usr/bin/env python3
"""Per-kernel table of any rocprofv3 --pmc counters (several passes merged by kernel name).

Every counter is averaged per dispatch of the kernel. Columns named SQ_WAIT_* / SQ_ACTIVE_INST_* /
SQ_INST_CYCLES_* / SQ_BUSY_CYCLES are also shown as a share of SQ_WAVE_CYCLES of the same pass
(both count quad-cycles summed over waves), SQ_LDS_BANK_CONFLICT / SQ_LDS_UNALIGNED_STALL /
SQ_LDS_ADDR_CONFLICT as a share of SQ_LDS_IDX_ACTIVE, and SQ_VALU_MFMA_BUSY_CYCLES as MFMA
utilisation = busy / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs).

  python tools/pmc_table.py --match hconv3,hwgrad2 pass1.csv pass2.csv ...
"""
import argparse
import csv
import re
from collections import defaultdict

SHARE_OF_WAVE = ("SQ_WAIT_", "SQ_ACTIVE_INST_", "SQ_INST_CYCLES_", "SQ_BUSY_CYCLES")
SHARE_OF_LDS = ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_UNALIGNED_STALL", "SQ_LDS_ADDR_CONFLICT")


def load(path):
    per = defaultdict(lambda: defaultdict(float))
    for d in csv.DictReader(open(path)):
        name = re.sub(r"\(.*$", "", d.get("Kernel_Name", d.get("Kernel-Name", "?")))
        name = re.sub(r"^void ", "", name)[:60]
        disp = d.get("Dispatch_Id", d.get("Dispatch-Id", "0"))
        per[(name, disp)][d.get("Counter_Name", d.get("Counter-Name"))] += float(
            d.get("Counter_Value", d.get("Counter-Value", 0)))
    out = defaultdict(lambda: defaultdict(list))
    for (name, _), cs in per.items():
        for k, v in cs.items():
            out[name][k].append(v)
    return {n: {k: sum(v) / len(v) for k, v in cs.items()} for n, cs in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="", help="comma-separated kernel-name substrings to keep")
    ap.add_argument("--wide", default="", help="one row per kernel with these comma-separated columns")
    a = ap.parse_args()
    keep = [m for m in a.match.split(",") if m]
    rows = defaultdict(dict)
    for path in a.csv:
        for name, cs in load(path).items():
            if keep and not any(k in name for k in keep):
                continue
            wc = cs.get("SQ_WAVE_CYCLES")
            lds = cs.get("SQ_LDS_IDX_ACTIVE")
            gui = cs.get("GRBM_GUI_ACTIVE")
            for k, v in cs.items():
                if k in ("SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE", "SQ_LDS_IDX_ACTIVE"):
                    rows[name].setdefault(k, f"{v:.3g}")
                elif k == "SQ_VALU_MFMA_BUSY_CYCLES" and gui:
                    rows[name]["MFMA util"] = f"{100 * v / (gui / 8 * 1024):.1f}%"
                elif k.startswith(SHARE_OF_WAVE) and wc:
                    rows[name][k.replace("SQ_", "")] = f"{100 * v / wc:.1f}%"
                elif k in SHARE_OF_LDS and lds:
                    rows[name][k.replace("SQ_", "") + "/LDS_ACTIVE"] = f"{100 * v / lds:.1f}%"
                else:
                    rows[name][k.replace("SQ_", "")] = f"{v:.4g}"
    if a.wide:
        cols_w = a.wide.split(",")
        print("| kernel | " + " | ".join(cols_w) + " |")
        print("|---|" + "---:|" * len(cols_w))
        for name, cols in sorted(rows.items()):
            print(f"| `{name}` | " + " | ".join(cols.get(c, "-") for c in cols_w) + " |")
        return
    for name, cols in sorted(rows.items()):
        print(f"### `{name}`\n")
        print("| counter | value |\n|---|---:|")
        for k in sorted(cols):
            print(f"| {k} | {cols[k]} |")
        print()


if __name__ == "__main__":
    main()
