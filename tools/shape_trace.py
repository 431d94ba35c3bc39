"""Per-launch shape table of one training step: the DFCSA_SHAPELOG lines of an eager bench run
(host call order) matched to the conv / wgrad kernels of its rocprofv3 kernel trace in dispatch
order (one kernel per conv launch; a wgrad launch is its GEMM kernel plus, with splits > 1 and
no fused reduction, one wgrad_reduce kernel).  The last complete step (delimited by clip_sgd) is
reported with flop/s per launch.
usage: python tools/shape_trace.py <run_results.db> <stderr log with SHAPE lines>"""
import re
import sqlite3
import sys


def main():
    db, log = sys.argv[1], sys.argv[2]
    shapes = [l.split(None, 2)[1:] for l in open(log) if l.startswith("SHAPE ")]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, duration, grid_x, workgroup_x, dispatch_id from kernels order by dispatch_id"))
    conv_k = ("conv_gemm_glds_kernel", "conv_gemm_kernel", "conv_gemm_pp_kernel", "conv1x1_stream_kernel",
              "conv_halo_kernel", "small_conv_f32_kernel")
    wg_k = ("wgrad_glds_kernel", "wgrad_kernel", "wgrad_halo_kernel", "small_wgrad_f32_kernel", "wgrad_simple")
    seq = []
    for name, d, gx, wx, did in rows:
        short = name.replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0]
        if short.startswith(conv_k):
            seq.append(("conv", short, d, gx // max(wx, 1)))
        elif short.startswith(wg_k):
            seq.append(("wgrad", short, d, gx // max(wx, 1)))
        elif short.startswith("wgrad_reduce"):
            seq.append(("reduce", short, d, gx // max(wx, 1)))
        elif short.startswith("clip_sgd"):
            seq.append(("step", short, d, 0))
    # walk kernels and shapes together
    out, si = [], 0
    i = 0
    while i < len(seq) and si < len(shapes):
        kind, short, d, g = seq[i]
        if kind == "step":
            out.append(("STEP",))
            i += 1
            continue
        fam, rest = shapes[si]
        if fam != kind:
            i += 1       # a kernel without a logged shape (fused block GEMMs share some names)
            continue
        red = 0
        if kind == "wgrad" and i + 1 < len(seq) and seq[i + 1][0] == "reduce":
            red = seq[i + 1][2]
            i += 1
        out.append((kind, short, d, g, rest.strip(), red))
        si += 1
        i += 1
    # last complete step
    idx = [k for k, r in enumerate(out) if r[0] == "STEP"]
    step = out[idx[-2] + 1: idx[-1]] if len(idx) >= 2 else out
    tot = 0.0
    for r in step:
        kind, short, d, g, rest, red = r
        kv = dict(p.split("=") for p in rest.split())
        if kind == "conv":
            fl = 2.0 * int(kv["M"]) * int(kv["N"]) * int(kv["K"])
        else:
            fl = 2.0 * int(kv["M"]) * int(kv["NI"]) * int(kv["NJ"])
        us = (d + red) / 1e3
        tot += us
        print(f"{us:8.1f} us {fl / (us * 1e-6) / 1e12:7.1f} TF  {short[:48]:48s} g={g:5d} red={red / 1e3:5.1f}  {rest}")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
