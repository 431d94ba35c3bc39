# 32-deep-slot ring tile (configs 30-35) vs the default and 64-deep tiles on the model's shapes;
# GEMM_CHECK: outputs compared with the first config (same MFMA order: expected bit-identical).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
GEMM_CHECK=1 timeout -k 10 600 python3 tools/gemm_bench.py 14,30,31,32,35,34,0 > gpurun_out/glds32.jsonl 2> gpurun_out/glds32.err
echo rc=$?
