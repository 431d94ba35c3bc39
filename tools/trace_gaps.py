"""Critical-path view of a rocprofv3 kernel trace (run_results.db): per training step (between
consecutive clip_sgd launches) the wall time, the union of kernel busy intervals, the idle gaps,
and the busy time by kernel name (overlap counted once per kernel)."""
import sqlite3, sys, collections
db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
clip = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
steps = []
for a, b in zip(clip[-6:-1], clip[-5:]):
    seg = rows[a + 1:b + 1]
    t0, t1 = seg[0][1], seg[-1][2]
    busy = 0; cur_s, cur_e = None, None; gaps = []
    for _, s, e in seg:
        if cur_e is None: cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s; gaps.append(s - cur_e); cur_s, cur_e = s, e
        else: cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    conc = sum(e - s for _, s, e in seg)
    steps.append((t1 - t0, busy, len(seg), sum(gaps), len(gaps), conc))
for w, b, n, g, ng, conc in steps:
    print(f"step wall {w/1e6:.3f} ms  busy(union) {b/1e6:.3f}  idle {g/1e6:.3f} ms in {ng} gaps  launches {n}  sum-of-kernels {conc/1e6:.3f}")
