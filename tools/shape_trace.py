"""Per-launch shape table of one training step: the DFCSA_SHAPELOG lines of an eager bench run
(host call order) matched to the conv / wgrad kernels of its rocprofv3 kernel trace in dispatch
order (one tile kernel per conv launch, plus its split-K epilogue launch when split; a wgrad launch
is its GEMM kernel plus its reduction / bias-sum launches).  The fused block GEMMs (gate / fusion
prologues and epilogues) and the one-launch LSA projection backward do not log a shape and are not
in the table.  The last complete step (delimited by clip_sgd) is reported.

Columns: time (us, GEMM + its reduction), TFLOP/s and its fraction of the dense MFMA peak (2.5
PFLOP/s bf16, 157 TFLOP/s fp32), algorithmic HBM bytes (unique input + weights + output; the 3x3
taps re-read one input, so the input counts once), TB/s and its fraction of 8 TB/s, and the bound
(whichever fraction a launch would hit first at full speed: flops / peak vs bytes / 8 TB/s).
usage: python tools/shape_trace.py <run_results.db> <stderr log with SHAPE lines>"""
import sqlite3
import sys

PEAK = {1: 2.5e15, 0: 157e12}
HBM = 8e12
CONV_K = ("conv_gemm_glds_kernel", "conv_gemm_glds32_kernel", "conv_gemm_kernel", "conv_gemm_pp_kernel",
          "conv1x1_stream_kernel", "conv_halo_kernel", "small_conv_f32_kernel")
WG_K = ("wgrad_bd_kernel", "wgrad_glds_kernel", "wgrad_kernel", "wgrad_halo_kernel", "small_wgrad_f32_kernel",
        "wgrad_simple")
RED_K = ("wgrad_reduce", "slab_colsum", "conv_splitk_epi")


def classify(short):
    if short.startswith(CONV_K):
        return "conv"
    if short.startswith(WG_K):
        return "wgrad"
    if short.startswith(RED_K):
        return "reduce"
    if short.startswith("clip_sgd"):
        return "step"
    return None


def distinct(nseg):
    """input re-read factor: 3x3 taps (9 per source) and the 9 + 2 segment dgrad read one tensor"""
    if nseg == 11:
        return 11
    if nseg % 9 == 0:
        return 9
    return 1


def algo_bytes(kind, kv):
    e = 2 if kv["dt"] == "1" else 4
    M = int(kv["M"])
    if kind == "conv":
        N, K, Kpad = int(kv["N"]), int(kv["K"]), int(kv["Kpad"])
        out = M * N * e * (2 if kv.get("acc") == "1" else 1)
        return M * K * e // distinct(int(kv["nseg"])) + N * Kpad * e + out
    NI, NJ = int(kv["NI"]), int(kv["NJ"])
    return M * NI * e + M * NJ * e // distinct(int(kv["nseg"])) + NI * NJ * 4


def main():
    db, log = sys.argv[1], sys.argv[2]
    shapes = [l.split(None, 2)[1:] for l in open(log) if l.startswith("SHAPE ")]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, duration, grid_x, workgroup_x, dispatch_id from kernels order by dispatch_id"))
    seq = []
    for name, d, gx, wx, did in rows:
        short = name.replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0]
        kind = classify(short)
        if kind:
            seq.append((kind, short, d, gx // max(wx, 1)))
    out, si, i = [], 0, 0
    while i < len(seq) and si < len(shapes):
        kind, short, d, g = seq[i]
        if kind == "step":
            out.append(("STEP",))
            i += 1
            continue
        if kind == "reduce":   # a reduction whose GEMM logged no shape (fused paths)
            i += 1
            continue
        fam, rest = shapes[si]
        if fam != kind:
            i += 1
            continue
        red = 0
        while i + 1 < len(seq) and seq[i + 1][0] == "reduce":
            red += seq[i + 1][2]
            i += 1
        out.append((kind, short, d, g, rest.strip(), red))
        si += 1
        i += 1
    idx = [k for k, r in enumerate(out) if r[0] == "STEP"]
    step = out[idx[-2] + 1: idx[-1]] if len(idx) >= 2 else out
    print(f"{'us':>8s} {'TF/s':>7s} {'mfma':>5s} {'MB':>7s} {'TB/s':>5s} {'hbm':>5s} {'bound':5s}  "
          f"{'kernel':44s} {'grid':>5s} {'red_us':>6s}  shape")
    tot = fl_tot = by_tot = 0.0
    for r in step:
        kind, short, d, g, rest, red = r
        kv = dict(p.split("=") for p in rest.split())
        if kind == "conv":
            fl = 2.0 * int(kv["M"]) * int(kv["N"]) * int(kv["K"])
        else:
            fl = 2.0 * int(kv["M"]) * int(kv["NI"]) * int(kv["NJ"])
        by = algo_bytes(kind, kv)
        us = (d + red) / 1e3
        tot += us
        fl_tot += fl
        by_tot += by
        peak = PEAK[int(kv["dt"])]
        fm = fl / (us * 1e-6) / peak
        fh = by / (us * 1e-6) / HBM
        bound = "mfma" if fl / peak >= by / HBM else "hbm"
        print(f"{us:8.1f} {fl / (us * 1e-6) / 1e12:7.1f} {fm:5.2f} {by / 1e6:7.1f} {by / (us * 1e-6) / 1e12:5.2f} "
              f"{fh:5.2f} {bound:5s}  {short[:44]:44s} {g:5d} {red / 1e3:6.1f}  {kind} {rest}")
    print(f"total {tot:.1f} us over {len(step)} launches: {fl_tot / 1e12:.3f} TFLOP, {by_tot / 1e9:.2f} GB algorithmic")


if __name__ == "__main__":
    main()
