#!/usr/bin/env python3
"""Hot-path purity check on a rocprofv3 trace of bench.py: in the LAST traced training step
(between the last two optimizer kernels, i.e. a steady-state graph replay) count ATen kernels and
copy/fill kernels. Every compute kernel of the step should be the framework's own (dcnn::...);
the only copies should be the input batch's two slots (images, labels).

  python tools/check_hot_path.py gpurun_out/prof_x/run_results.db [--max-copies 2]
Exit status 1 when the step has an ATen kernel or more copies than allowed.
"""
import re
import sqlite3
import sys


def main():
    path = sys.argv[1]
    max_copies = int(sys.argv[sys.argv.index("--max-copies") + 1]) if "--max-copies" in sys.argv else 2
    c = sqlite3.connect(path)
    rows = [r[0] for r in c.execute("select name from kernels order by start")]
    opt = [i for i, n in enumerate(rows) if "adam_kernel" in n or "sgd_kernel" in n]
    if len(opt) < 2:
        sys.exit("need two optimizer dispatches in the trace")
    step = rows[opt[-2] + 1:opt[-1] + 1]
    aten = [n for n in step if "at::" in n]
    copies = [n for n in step if "copyBuffer" in n]
    fills = [n for n in step if "fillBuffer" in n]
    ours = [n for n in step if "dcnn" in n]
    print(f"kernels in the last step: {len(step)}; framework (dcnn::) {len(ours)}; ATen {len(aten)}; "
          f"copies {len(copies)}; memset fills {len(fills)}")
    for n in sorted(set(aten)):
        print("  ATen:", re.sub(r"\(.*", "", n)[:100])
    ok = not aten and len(copies) <= max_copies
    print("hot path: PURE" if ok else "hot path: NOT pure")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
