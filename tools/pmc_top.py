"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE x2 gfx950 correction)."""
import sqlite3, collections, sys
def per_kernel(db, counter):
    c = sqlite3.connect(db)
    out = collections.defaultdict(lambda: [0, 0.0])
    for name, v in c.execute("select kernel_name, sum(value) from counters_collection where counter_name=? "
                             "group by dispatch_id", (counter,)):
        out[name][0] += 1
        out[name][1] += v * 1024
    return out
f = per_kernel(sys.argv[1], "FETCH_SIZE")
w = per_kernel(sys.argv[2], "WRITE_SIZE")
for k in sorted(f, key=lambda k: -f[k][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 12]:
    n, b = f[k]
    nw, bw = w.get(k, [1, 0])
    print(f"{k.replace('(anonymous namespace)::', '')[:64]:64s} n={n:4d} read/launch {2 * b / n / 1e6:8.2f} MB "
          f"write/launch {bw / max(nw, 1) / 1e6:8.2f} MB")
