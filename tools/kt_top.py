"""Top kernels of the replayed bench step from a rocprofv3 kernel-trace database (the last `steps`
clip_sgd-delimited steps): average time per step and launches per step, by kernel name.

  python tools/kt_top.py run_results.db [steps] [top]
"""
import re
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    ends = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
    sel = rows[ends[-steps - 1] + 1: ends[-1] + 1]
    per = defaultdict(lambda: [0, 0.0])
    for n, s, e in sel:
        k = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:72]
        per[k][0] += 1
        per[k][1] += (e - s) / 1e3
    wall = (sel[-1][2] - sel[0][1]) / 1e6 / steps
    print(f"{db}: {len(sel) / steps:.0f} launches/step, first-to-last kernel {wall:.2f} ms/step")
    for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {t / steps:8.1f} us {n / steps:5.1f}x  {k}")


if __name__ == "__main__":
    main()
