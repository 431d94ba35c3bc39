mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
GEMM_SHAPES="L2 3x3,L3 3x3,L4 3x3 dgrad up" timeout -k 10 400 python -u tools/gemm_bench.py 14,22,0,14,22,0 > gpurun_out/gemm_cfgs2.jsonl 2>&1
