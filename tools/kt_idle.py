"""Where the chip is under-filled in a bench step (rocprofv3 kernel trace): sweeps one step's kernels
over time and sums the time during which the running kernels' workgroups total fewer than
`--min` (default 256) -- a latency-bound stretch -- attributing it to the kernels running then.

  python tools/kt_idle.py run_results.db [min_wgs]
"""
import re
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    mn = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, grid_x / workgroup_x * grid_y / workgroup_y * grid_z / workgroup_z, start, end "
                          "from kernels order by start"))
    b = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
    nst = 5
    blame = defaultdict(float)
    tot_idle = tot_gap = 0.0
    for k in range(-nst - 1, -1):
        st = rows[b[k] + 1:b[k + 1] + 1]
        ev = []
        for i, (n, g, t0, t1) in enumerate(st):
            ev.append((t0, 1, i))
            ev.append((t1, -1, i))
        ev.sort()
        active = set()
        last = ev[0][0]
        for t, d, i in ev:
            dt = (t - last) / 1e3
            if dt > 0:
                wgs = sum(st[j][1] for j in active)
                if not active:
                    tot_gap += dt
                elif wgs < mn:
                    tot_idle += dt
                    for j in active:
                        nm = re.sub(r"\(.*", "", st[j][0].replace("(anonymous namespace)::", "").replace("void ", ""))[:55]
                        blame[nm] += dt / len(active)
            last = t
            if d > 0:
                active.add(i)
            else:
                active.discard(i)
    print(f"per step: under-filled (< {mn} WGs) {tot_idle / nst:.1f} us, nothing running {tot_gap / nst:.1f} us")
    for nm, v in sorted(blame.items(), key=lambda x: -x[1])[:30]:
        print(f"{v / nst:8.1f} us  {nm}")


if __name__ == "__main__":
    main()
