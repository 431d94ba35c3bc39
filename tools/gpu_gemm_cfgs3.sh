mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
GEMM_SHAPES="BN 3x3,L4 3x3,L3 3x3 dgrad down3" timeout -k 10 400 python -u tools/gemm_bench.py 0,19,3,12,15,0,19 > gpurun_out/gemm_cfgs3.jsonl 2>&1
