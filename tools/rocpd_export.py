"""Turn rocprofv3 SQLite outputs (run_results.db) into the committed profile summaries.

  python tools/rocpd_export.py stats  <kernel-trace db> <out.csv>
      per-kernel Name,Calls,TotalDurationNs,AverageNs,Percentage (the --stats layout)
  python tools/rocpd_export.py classes <kernel-trace db> <out.json>
      launches / average duration of the bench's roofline kernel classes
  python tools/rocpd_export.py traffic <FETCH_SIZE db> <WRITE_SIZE db> <out.json>
      HBM bytes per dispatch of the kernels whose name contains `pattern` (default conv_gemm),
      corrected as /opt/skills/guides/MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE and
      WRITE_SIZE are kilobytes; FETCH_SIZE counts half the bytes of 16-B/lane streaming reads
      (x2), WRITE_SIZE is exact for 16-B/lane stores.  Each counter comes from its own pass.
"""
import csv
import json
import sqlite3
import sys
from collections import defaultdict


def stats(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration) from kernels group by name order by sum(duration) desc")
    rows = list(rows)
    tot = sum(r[2] for r in rows)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, n, d in rows:
            w.writerow([name, n, d, d / n, 100.0 * d / tot])


def classes(db, out):
    """Per kernel class (the bench roofline classes): launches, total and average duration."""
    c = sqlite3.connect(db)
    res = {}
    for cls, pats in CLASSES.items():
        n, tot = 0, 0
        for name, cnt, d in c.execute("select name, count(*), sum(duration) from kernels group by name"):
            if any(p in name for p in pats):
                n += cnt
                tot += d
        res[cls] = {"launches": n, "total_ms": tot / 1e6, "avg_launch_ms": tot / 1e6 / max(n, 1)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


def _per_dispatch(db, counter):
    c = sqlite3.connect(db)
    out = {}
    for did, name, val in c.execute("select dispatch_id, kernel_name, sum(value) from counters_collection "
                                    "where counter_name = ? group by dispatch_id", (counter,)):
        out[did] = (name, val * 1024.0)
    return out


CLASSES = {"conv_gemm": ("conv_gemm_glds_kernel", "conv_gemm_kernel<"),
           "conv_wgrad": ("wgrad_glds_kernel", "wgrad_kernel<"),
           "conv1x1_stream": ("conv1x1_stream_kernel",)}


def traffic(fdb, wdb, out, pattern="conv_gemm"):
    fetch = _per_dispatch(fdb, "FETCH_SIZE")
    write = _per_dispatch(wdb, "WRITE_SIZE")
    per_kernel = defaultdict(lambda: {"launches_fetch": 0, "read_bytes": 0.0, "launches_write": 0, "write_bytes": 0.0})
    for name, v in fetch.values():
        k = per_kernel[name]
        k["launches_fetch"] += 1
        k["read_bytes"] += 2.0 * v          # gfx950 FETCH_SIZE = 1/2 of streamed bytes
    for name, v in write.values():
        k = per_kernel[name]
        k["launches_write"] += 1
        k["write_bytes"] += v
    pats = CLASSES.get(pattern, (pattern,))
    sel = {n: k for n, k in per_kernel.items() if any(p in n for p in pats)}
    nf = sum(k["launches_fetch"] for k in sel.values())
    nw = sum(k["launches_write"] for k in sel.values())
    rd = sum(k["read_bytes"] for k in sel.values())
    wr = sum(k["write_bytes"] for k in sel.values())
    res = {"class": pattern, "kernels": list(pats), "launches": nf,
           "hbm_bytes_per_launch": (rd / max(nf, 1)) + (wr / max(nw, 1)),
           "read_bytes_per_launch": rd / max(nf, 1), "write_bytes_per_launch": wr / max(nw, 1),
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB",
           "per_kernel": {n: {"launches": k["launches_fetch"],
                              "read_MB_per_launch": k["read_bytes"] / max(k["launches_fetch"], 1) / 1e6,
                              "write_MB_per_launch": k["write_bytes"] / max(k["launches_write"], 1) / 1e6}
                          for n, k in sorted(sel.items(), key=lambda kv: -kv[1]["read_bytes"])}}
    return res


def traffic_all(fdb, wdb, out):
    res = {c: traffic(fdb, wdb, None, c) for c in CLASSES}
    json.dump(res, open(out, "w"), indent=1)
    for c, r in res.items():
        print(c, r["launches"], round(r["hbm_bytes_per_launch"] / 1e6, 2), "MB/launch")


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "classes":
        classes(sys.argv[2], sys.argv[3])
    else:
        traffic_all(*sys.argv[2:5])
