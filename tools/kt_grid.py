"""Median duration per launch grid of the kernels matching a name pattern in one or two
rocprofv3 kernel-trace databases:  python tools/kt_grid.py <pattern> <db> [<db2>]"""
import sqlite3
import sys
from collections import defaultdict

pat = sys.argv[1]
for db in sys.argv[2:]:
    c = sqlite3.connect(db)
    d = defaultdict(list)
    for name, dur, gx, gy, gz, wx in c.execute(
            "select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels where name like ?",
            ("%" + pat + "%",)):
        d[(name.replace("(anonymous namespace)::", "")[:48], gx // wx, gy, gz, wx)].append(dur)
    print(db)
    for k, v in sorted(d.items()):
        v.sort()
        print(f"  {k[0]:48s} grid {k[1]:6d}x{k[2]:4d}x{k[3]:3d} wg {k[4]:4d}  n {len(v):5d}  med {v[len(v) // 2] / 1e3:8.2f} us")
