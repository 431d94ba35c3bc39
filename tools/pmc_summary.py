"""Per-kernel PMC summary of rocprofv3 counter databases (run_results.db), one line per kernel
(name pattern) with each counter's value averaged over its dispatches, plus derived ratios.

  python tools/pmc_summary.py <pattern> <db> [<db> ...]
"""
import sqlite3
import sys
from collections import defaultdict


def collect(pattern, dbs):
    vals = defaultdict(list)
    meta = {}
    for db in dbs:
        c = sqlite3.connect(db)
        rows = c.execute("select dispatch_id, kernel_name, counter_name, value, vgpr_count, accum_vgpr_count, "
                         "lds_block_size, grid_size, workgroup_size from counters_collection")
        per = defaultdict(float)
        for d, name, cn, v, vg, ag, lds, gs, ws in rows:
            if pattern not in name:
                continue
            per[(d, cn)] += v           # summed over the dimensions of one dispatch
            meta = {"vgpr": vg, "agpr": ag, "lds": lds, "grid": gs, "wg": ws, "name": name[:90]}
        for (d, cn), v in per.items():
            vals[cn].append(v)
    return {k: sum(v) / len(v) for k, v in vals.items()}, meta


def main():
    pat, dbs = sys.argv[1], sys.argv[2:]
    avg, meta = collect(pat, dbs)
    print(meta)
    for k in sorted(avg):
        print(f"  {k:32s} {avg[k]:.4g}")
    g = avg.get
    if g("SQ_WAVE_CYCLES"):
        wc = g("SQ_WAVE_CYCLES")
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if g(k):
                print(f"  {k} / WAVE_CYCLES = {g(k) / wc:.3f}")
    if g("SQ_LDS_BANK_CONFLICT") and g("SQ_LDS_IDX_ACTIVE"):
        print(f"  LDS conflict share = {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
    if g("SQ_INSTS_VALU") and g("SQ_INSTS_MFMA"):
        print(f"  VALU per MFMA = {g('SQ_INSTS_VALU') / g('SQ_INSTS_MFMA'):.2f}")
    if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
        print(f"  MFMA busy (per SIMD) = {g('SQ_VALU_MFMA_BUSY_CYCLES') / (g('GRBM_GUI_ACTIVE') / 8 * 1024):.3f}")


if __name__ == "__main__":
    main()
