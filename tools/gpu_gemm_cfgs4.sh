mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
GEMM_SHAPES="L1 3x3 fwd,L2 3x3 dgrad N64" timeout -k 10 400 python -u tools/gemm_bench.py 17,11,4,3,12,17 > gpurun_out/gemm_cfgs4.jsonl 2>&1
