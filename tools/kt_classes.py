"""Per-class kernel time of one bench step from a rocprofv3 kernel trace, split by queue (the main
compute queue is the critical path; the branch stream's kernels overlap it).

  python tools/kt_classes.py run_results.db
"""
import re
import sqlite3
import sys
from collections import defaultdict

CLASSES = [("wgrad_reduce", r"wgrad_reduce"), ("wgrad", r"wgrad"), ("conv_gemm", r"conv_gemm_glds|conv_gemm_pp|splitk_epi|conv_gemm_kernel|conv_halo"),
           ("fused_block_gemm", r"dgrad_gate|gate_fusion_fwd"), ("conv1x1_stream", r"conv1x1_stream"),
           ("ew_red", r"ew_red"), ("ew_fwd", r"ew_fwd"), ("bn_finalize", r"bn_finalize|bn_bwd_finalize|slab_colsum|colred"),
           ("lsa", r"lsa_|small_conv_f32|small_wgrad_f32"), ("block_out/pool", r"block_out|maxpool"),
           ("optimizer", r"clip_sgd|sumsq"), ("pack", r"pack_plan|pack_"), ("loss/head", r"bce|sigmoid|head")]


def classify(n):
    for c, rx in CLASSES:
        if re.search(rx, n):
            return c
    return "other:" + re.sub(r"\(.*|<.*", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:40]


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = list(c.execute("select name, start, end, queue_id from kernels order by start"))
    b = [i for i, r in enumerate(rows) if "clip_sgd" in r[0]]
    steps = [rows[x + 1:y + 1] for x, y in zip(b[-11:-1], b[-10:])]
    per = defaultdict(float)
    cnt = defaultdict(float)
    main_q = max(set(r[3] for r in steps[0]), key=lambda q: sum(1 for r in steps[0] if r[3] == q))
    for st in steps:
        for n, t0, t1, q in st:
            k = (classify(n), "main" if q == main_q else "branch")
            per[k] += (t1 - t0) / 1e3 / len(steps)
            cnt[k] += 1 / len(steps)
    tot = defaultdict(float)
    for (k, q), v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"{v:9.1f} us  {cnt[(k, q)]:6.1f} launches  {q:6s} {k}")
        tot[q] += v
    print({q: round(v, 1) for q, v in tot.items()})


if __name__ == "__main__":
    main()
