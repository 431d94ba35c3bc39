# Round 5, TransUNet (config 4): GroupNorm tests (fused and four-launch paths), the bf16 bench
# line, and the per-launch GEMM shape table of one eager step (streams serialised).
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_transunet.py -k "groupnorm" -q -x --timeout 120 --timeout-method thread > gpurun_out/tu_gn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tu_gn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
S="--model transunet --batch 8 --precision bf16 --no-cpu-baseline --no-val-dice --no-trainer-faithful"
timeout -k 10 300 python bench.py $S --steps 10 --warmup 3 > gpurun_out/tu_bench.json 2> gpurun_out/tu_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/tu_s_trace
export DFCSA_SHAPELOG=1 DFCSA_SIDE_STREAM=0 DFCSA_BRANCH_STREAM=0
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tu_s_trace -o run -- python3 $R/bench.py $S --steps 2 --warmup 1 --no-graph --no-kernel-timing > $R/gpurun_out/tu_s_trace.out 2> $R/gpurun_out/tu_s_trace.err || exit 1
unset DFCSA_SHAPELOG DFCSA_SIDE_STREAM DFCSA_BRANCH_STREAM
cd $R
DB=$(ls gpurun_out/tu_s_trace/*/run_results.db gpurun_out/tu_s_trace/run_results.db 2>/dev/null | head -1)
python3 tools/shape_trace.py $DB gpurun_out/tu_s_trace.err > gpurun_out/tu_shape_trace.txt 2>&1
echo done
