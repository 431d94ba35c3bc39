"""One training step's kernels from a rocprofv3 kernel-trace database, in launch order, grouped
by (kernel, grid): count and total/avg device time per step.  Steps are delimited by the
clip_sgd launches; the last complete step is analysed.
usage: python tools/step_kernels.py <run_results.db> [top]"""
import sqlite3
import sys
from collections import OrderedDict


def main():
    db, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, duration, start, end from kernels order by start"))
    ends = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
    step = rows[ends[-2] + 1: ends[-1] + 1]
    wall = (step[-1][7] - step[0][6]) / 1e6
    busy = sum(r[5] for r in step) / 1e6
    agg = OrderedDict()
    for name, gx, gy, gz, wx, d, _, _ in step:
        short = name.replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0]
        k = (short[:70], f"{gx // max(wx, 1)}x{gy}x{gz}/{wx}")
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += d / 1e3
    print(f"launches {len(step)}  device-busy {busy:.3f} ms  first->last wall {wall:.3f} ms  gaps {wall - busy:.3f} ms")
    for (n, g), (cnt, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{us:9.1f} us  {cnt:3d}x  {us / cnt:8.1f} us  {g:18s} {n}")


if __name__ == "__main__":
    main()
