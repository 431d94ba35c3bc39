"""Turn rocprofv3 SQLite outputs (run_results.db) into the committed profile summaries.

  python tools/rocpd_export.py stats  <kernel-trace db> <out.csv>
      per-kernel Name,Calls,TotalDurationNs,AverageNs,Percentage (the --stats layout)
  python tools/rocpd_export.py classes <kernel-trace db> <out.json>
      launches / average duration of the bench's roofline kernel classes
  python tools/rocpd_export.py step <FETCH_SIZE db> <WRITE_SIZE db> <out.json>
      HBM bytes of ONE whole training step (the dispatches after the second-to-last clip_sgd
      launch up to the last one) in total and per kernel group (bench.py's step_roofline.hbm_frac)
  python tools/rocpd_export.py replay <kernel-trace db> <out.json> [steps]
      per roofline class and per kernel group: launches and kernel time per step over the LAST
      `steps` (default 5) complete steps of the trace, split at the clip_sgd launches -- with
      `bench.py --no-kernel-timing ...` under rocprofv3 these are the timed HIP-graph replays, every
      stream concurrent (bench.py's roofline.replayed reads it)
  python tools/rocpd_export.py sq <SQ/GRBM counter db> <out.json>
      per kernel group: SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_MFMA, SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE,
      GRBM_GUI_ACTIVE and the MFMA-busy fraction = MFMA busy cycles / (GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
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


def replay(db, out, steps=5):
    """Class and group kernel time of the replayed step (last `steps` steps, clip_sgd-delimited)."""
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    ends = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
    if len(ends) < steps + 1:
        raise SystemExit(f"need >= {steps + 1} clip_sgd launches in the trace, found {len(ends)}")
    sel = rows[ends[-steps - 1] + 1: ends[-1] + 1]
    wall = (sel[-1][2] - sel[0][1]) / 1e6 / steps
    res = {"steps": steps, "launches_per_step": len(sel) / steps, "first_to_last_kernel_ms_per_step": wall,
           "definition": "kernel durations (end - start) summed per class / group over the last `steps` "
                         "clip_sgd-delimited steps, divided by `steps`; concurrent streams overlap, so the "
                         "sum over groups exceeds the wall time", "classes": {}, "groups": {}}
    for cls, pats in CLASSES.items():
        ks = [r for r in sel if any(p in r[0] for p in pats)]
        res["classes"][cls] = {"launches_per_step": len(ks) / steps,
                               "ms_per_step": sum(r[2] - r[1] for r in ks) / 1e6 / steps}
    grp = defaultdict(lambda: [0, 0])
    for n, s_, e_ in sel:
        g = grp[group_of(n)]
        g[0] += 1
        g[1] += e_ - s_
    res["groups"] = {k: {"launches_per_step": v[0] / steps, "ms_per_step": v[1] / 1e6 / steps}
                     for k, v in sorted(grp.items(), key=lambda kv: -kv[1][1])}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["classes"]), round(wall, 3), "ms first-to-last kernel per step")


def _per_dispatch(db, counter):
    c = sqlite3.connect(db)
    out = {}
    for did, name, val in c.execute("select dispatch_id, kernel_name, sum(value) from counters_collection "
                                    "where counter_name = ? group by dispatch_id", (counter,)):
        out[did] = (name, val * 1024.0)
    return out


CLASSES = {"conv_gemm": ("conv_gemm_glds_kernel", "conv_gemm_kernel<", "conv_gemm_pp_kernel", "conv_halo_kernel",
                         "conv_gemm_glds32_kernel", "conv_splitk_epi_kernel", "conv_gemm_ppsk_kernel",
                         "small_conv_f32_kernel"),
           "conv_wgrad": ("wgrad_glds_kernel", "wgrad_bd_kernel", "wgrad_kernel<", "wgrad_halo_kernel"),
           # bench.py's class 4 (DFCSA_PROF_CONV_STREAM) times the streaming 1x1 GEMMs AND the fused
           # block GEMMs (dfcsa_dgrad_gate*, dfcsa_gate_fusion_fwd, dfcsa_local_attn_gate_fwd): the
           # same union here, so roofline.traffic matches the timed launches; the fused ones alone
           # as fused_block_gemm
           "conv1x1_stream": ("conv1x1_stream_kernel", "dgrad_gate_kernel", "gate_fusion_fwd_kernel"),
           "fused_block_gemm": ("dgrad_gate_kernel", "gate_fusion_fwd_kernel")}


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


GROUPS = (("conv_gemm", ("conv_gemm_glds_kernel", "conv_gemm_kernel<", "conv_gemm_pp_kernel", "conv_halo_kernel",
                         "small_conv_f32_kernel", "conv_gemm_glds32_kernel", "conv_splitk_epi_kernel",
                         "conv_gemm_ppsk_kernel")),
          ("conv_wgrad", ("wgrad_glds_kernel", "wgrad_bd_kernel", "wgrad_kernel<", "wgrad_halo_kernel",
                          "wgrad_reduce", "small_wgrad_f32_kernel", "small_wgrad_dgrad_f32_kernel")),
          ("conv1x1_stream", ("conv1x1_stream_kernel",)),
          ("fused_block_gemm (1x1 GEMMs with the gate / BN prologues and epilogues)",
           ("dgrad_gate_kernel", "gate_fusion_fwd_kernel")),
          ("block_out_pool (block output + max-pool fwd/bwd)", ("block_out_pool_kernel",)),
          ("ew_red (BN/gate/attention backward elementwise + partial sums)", ("ew_red_kernel", "ew_red_pair_kernel")),
          ("ew_fwd (BN apply, gate fusion, block output)", ("ew_fwd_kernel",)),
          ("bn_and_slab_finalizers", ("rows_reduce_kernel", "bn_finalize_kernel", "bn_bwd_finalize_kernel", "bn_bwd_finalize_pool",
                                      "slab_colsum", "sum_scalar_kernel", "colred")),
          ("lsa (pooled attention)", ("lsa_",)),
          ("maxpool", ("maxpool2",)),
          ("optimizer", ("sumsq_kernel", "clip_sgd")),
          ("pack_plan", ("pack_plan_kernel",)),
          ("loss/head/input", ("bce_dice", "sigmoid", "head_", "pack_input")))


def group_of(name):
    for g, pats in GROUPS:
        if any(p in name for p in pats):
            return g
    return "other"


def _dispatch_rows(db, counter):
    c = sqlite3.connect(db)
    return list(c.execute("select dispatch_id, kernel_name, sum(value) from counters_collection where counter_name = ? "
                          "group by dispatch_id order by dispatch_id", (counter,)))


def _last_step(rows):
    ends = [i for i, (_, n, _) in enumerate(rows) if "clip_sgd" in n]
    if len(ends) < 2:
        raise SystemExit("need >= 2 clip_sgd dispatches (2 steps) in the counter pass")
    return rows[ends[-2] + 1: ends[-1] + 1]


def step(fdb, wdb, out):
    rd = _last_step(_dispatch_rows(fdb, "FETCH_SIZE"))
    wr = _last_step(_dispatch_rows(wdb, "WRITE_SIZE"))
    groups = defaultdict(lambda: {"launches": 0, "read_bytes": 0.0, "write_bytes": 0.0})
    for _, n, v in rd:
        g = groups[group_of(n)]
        g["launches"] += 1
        g["read_bytes"] += 2.0 * v * 1024.0
    for _, n, v in wr:
        groups[group_of(n)]["write_bytes"] += v * 1024.0
    tot_r = sum(g["read_bytes"] for g in groups.values())
    tot_w = sum(g["write_bytes"] for g in groups.values())
    res = {"hbm_bytes_per_step": tot_r + tot_w, "read_bytes_per_step": tot_r, "write_bytes_per_step": tot_w,
           "launches_per_step": len(rd),
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB; one step = the "
                         "dispatches after the second-to-last clip_sgd launch through the last one",
           "groups": {k: {"launches": v["launches"], "read_MB": round(v["read_bytes"] / 1e6, 2),
                          "write_MB": round(v["write_bytes"] / 1e6, 2)}
                      for k, v in sorted(groups.items(), key=lambda kv: -(kv[1]["read_bytes"] + kv[1]["write_bytes"]))}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "groups"}))


def sq(db, out):
    c = sqlite3.connect(db)
    per = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    for did, name, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection "
                                      "group by dispatch_id, counter_name"):
        g = group_of(name)
        per[g][cn] += v
        launches[g].add(did)
    res = {}
    for g, d in per.items():
        r = {k: v for k, v in d.items()}
        r["launches"] = len(launches[g])
        if d.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            r["mfma_busy_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
        if d.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_bank_conflict_frac"] = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / d["SQ_LDS_IDX_ACTIVE"]
        if d.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in d:
            r["valu_per_mfma"] = d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"]   # SQ_INSTS_VALU counts the MFMAs too
        if d.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in d:
            r["wait_any_frac"] = d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
        res[g] = r
    res["_definition"] = ("mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs), "
                          "summed over the group's dispatches; lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / "
                          "SQ_LDS_IDX_ACTIVE; valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA (VALU includes the "
                          "MFMAs); wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES")
    json.dump(res, open(out, "w"), indent=1)
    for g, r in res.items():
        if g[0] != "_":
            print(g, r.get("launches"), round(r.get("mfma_busy_frac", float("nan")), 4))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "classes":
        classes(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "step":
        step(sys.argv[2], sys.argv[3], sys.argv[4])
    elif sys.argv[1] == "replay":
        replay(sys.argv[2], sys.argv[3], *(int(a) for a in sys.argv[4:5]))
    elif sys.argv[1] == "sq":
        sq(sys.argv[2], sys.argv[3])
    else:
        traffic_all(*sys.argv[2:5])
