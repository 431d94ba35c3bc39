"""Time per graph-replayed bench step during which ONLY kernels of a family run (e.g. only weight
gradients: the backward's main chain idle), from a rocprofv3 kernel trace.
  python tools/kt_only.py run_results.db 'wgrad' """
import re
import sqlite3
import sys


def main():
    db, pat = sys.argv[1], re.compile(sys.argv[2])
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    b = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
    tot = {"only": 0.0, "none": 0.0, "mixed": 0.0, "other": 0.0}
    nst = 5
    for k in range(-nst - 1, -1):
        st = rows[b[k] + 1:b[k + 1] + 1]
        ev = sorted([(s, 1, i) for i, (n, s, e) in enumerate(st)] + [(e, -1, i) for i, (n, s, e) in enumerate(st)])
        act, last = set(), ev[0][0]
        for t, d, i in ev:
            dt = (t - last) / 1e3
            if dt > 0:
                fam = [bool(pat.search(st[j][0])) for j in act]
                key = "none" if not fam else ("only" if all(fam) else ("mixed" if any(fam) else "other"))
                tot[key] += dt
            last = t
            (act.add if d > 0 else act.discard)(i)
    print({k: round(v / nst, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
