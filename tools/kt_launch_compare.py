"""Per-launch comparison of two rocprofv3 kernel traces of the bench step (arms A and B).

  python tools/kt_launch_compare.py A.db B.db [filter-regex]

Steps are delimited by the optimizer kernel (clip_sgd); the last 10 steps of each trace are kept.
Kernels are keyed by (name without template arguments' namespaces, grid size), the average
duration per step of each key is printed for both arms (keys matching the regex, default: all),
then the device-busy time and first->last span per step of both arms.
"""
import re
import sqlite3
import sys
from collections import defaultdict


def steps(db, keep=10):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, grid_x, start, end from kernels order by start"))
    bounds = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
    out = []
    for a, b in zip(bounds[-keep - 1:-1], bounds[-keep:]):
        out.append(rows[a + 1:b + 1])
    return out


def key(name, grid):
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))
    return f"{n[:70]} g={grid}"


def agg(st):
    per = defaultdict(float)
    cnt = defaultdict(int)
    busy = span = 0.0
    for s in st:
        for n, g, t0, t1 in s:
            per[key(n, g)] += (t1 - t0) / 1e3
            cnt[key(n, g)] += 1
            busy += (t1 - t0) / 1e3
        span += (s[-1][3] - s[0][2]) / 1e3
    k = len(st)
    return {x: v / k for x, v in per.items()}, {x: v / k for x, v in cnt.items()}, busy / k, span / k


def main():
    A, B = steps(sys.argv[1]), steps(sys.argv[2])
    rx = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    pa, ca, ba, sa = agg(A)
    pb, cb, bb, sb = agg(B)
    rows = []
    for k in set(pa) | set(pb):
        if rx and not rx.search(k):
            continue
        rows.append((pb.get(k, 0) - pa.get(k, 0), k))
    rows.sort()
    for d, k in rows:
        print(f"{d:+9.1f} us  A {pa.get(k, 0):8.1f} ({ca.get(k, 0):4.1f}x)  B {pb.get(k, 0):8.1f} ({cb.get(k, 0):4.1f}x)  {k}")
    print(f"per step: busy A {ba:.1f} us B {bb:.1f} us; first->last A {sa:.1f} us B {sb:.1f} us")


if __name__ == "__main__":
    main()
