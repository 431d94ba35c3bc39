# Streaming-GEMM change A/B: tests, the ConvTranspose / mid-M 1x1 shape bench on both libraries,
# then the step A/B (tools/gpu_r04_lib_ab.sh).
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
DFCSA_LIB=$R/$1 timeout -k 10 300 python tools/stream_minm_bench.py > gpurun_out/sm_base.jsonl 2>&1 || { tail gpurun_out/sm_base.jsonl; exit 1; }
timeout -k 10 300 python tools/stream_minm_bench.py > gpurun_out/sm_new.jsonl 2>&1 || { tail gpurun_out/sm_new.jsonl; exit 1; }
bash tools/gpu_r04_lib_ab.sh $1 "$2"
