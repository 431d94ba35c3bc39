mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 400 python -u tools/gemm_bench.py 0,5,6,10,13,14,16,18,22 > gpurun_out/gemm_cfgs.jsonl 2>&1
