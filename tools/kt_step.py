"""One graph-replayed bench step from a rocprofv3 kernel trace, per HW queue: kernel time, the
time with nothing running on the chip, and the time only one queue runs (critical-path view).

  python tools/kt_step.py run_results.db [--list]
"""
import re
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))
    return n[:60]


def steps(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, queue_id, start, end, grid_x/workgroup_x*grid_y/workgroup_y*grid_z/workgroup_z "
                          "from kernels order by start"))
    b = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
    return rows, b


def main():
    db = sys.argv[1]
    rows, b = steps(db)
    st = rows[b[-3] + 1:b[-2] + 1]
    t0 = st[0][2]
    q = defaultdict(float)
    for n, qi, s, e, g in st:
        q[qi] += (e - s) / 1e3
    wall = (st[-1][3] - t0) / 1e3
    print(f"step wall {wall:.1f} us, {len(st)} kernels; per queue kernel-us:", {k: round(v, 1) for k, v in q.items()})
    # sweep
    ev = sorted([(s, 1, i) for i, (n, qi, s, e, g) in enumerate(st)] + [(e, -1, i) for i, (n, qi, s, e, g) in enumerate(st)])
    active = set()
    last = ev[0][0]
    none = 0.0
    byset = defaultdict(float)
    for t, d, i in ev:
        dt = (t - last) / 1e3
        if dt > 0:
            qs = tuple(sorted({st[j][1] for j in active}))
            if not active:
                none += dt
            byset[qs] += dt
        last = t
        (active.add if d > 0 else active.discard)(i)
    print(f"nothing running: {none:.1f} us")
    for k, v in sorted(byset.items(), key=lambda x: -x[1]):
        print(f"  queues {k}: {v:.1f} us")
    if "--list" in sys.argv:
        for n, qi, s, e, g in st:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{qi} {g:6d} {short(n)}")


if __name__ == "__main__":
    main()
