"""Per-kernel comparison of two rocprofv3 kernel-trace databases (tools/gpu_ab_ktrace.sh).

  python tools/kt_compare.py <base run_results.db> <new run_results.db> [top]
prints, per kernel name (template arguments cut), calls and total / average duration in both
traces and the change of the total, sorted by |change|.
"""
import re
import sqlite3
import sys


def load(db):
    c = sqlite3.connect(db)
    out = {}
    for name, n, tot in c.execute("select name, count(*), sum(duration) from kernels group by name"):
        k = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))[:90]
        a = out.setdefault(k, [0, 0])
        a[0] += n
        a[1] += tot
    return out


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = []
    for k in set(a) | set(b):
        na, ta = a.get(k, (0, 0))
        nb, tb = b.get(k, (0, 0))
        rows.append((tb - ta, k, na, ta, nb, tb))
    rows.sort(key=lambda r: -abs(r[0]))
    ta_all = sum(v[1] for v in a.values())
    tb_all = sum(v[1] for v in b.values())
    print(f"total ms base {ta_all / 1e6:.2f} new {tb_all / 1e6:.2f} delta {(tb_all - ta_all) / 1e6:+.2f}")
    for d, k, na, ta, nb, tb in rows[:top]:
        avg_a = ta / na / 1e3 if na else 0
        avg_b = tb / nb / 1e3 if nb else 0
        print(f"{d / 1e6:+8.3f} ms  {na:6d} {avg_a:8.2f}us -> {nb:6d} {avg_b:8.2f}us  {k}")


if __name__ == "__main__":
    main()
