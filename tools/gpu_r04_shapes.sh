# Per-launch shapes of one eager step matched to a kernel trace (tools/shape_trace.py).
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/s_trace
export DFCSA_SHAPELOG=1 DFCSA_SIDE_STREAM=0 DFCSA_BRANCH_STREAM=0   # serial streams: standalone launch durations
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s_trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-graph --no-kernel-timing --no-cpu-baseline --no-val-dice --no-trainer-faithful > $R/gpurun_out/s_trace.out 2> $R/gpurun_out/s_trace.err || exit 1
unset DFCSA_SHAPELOG DFCSA_SIDE_STREAM DFCSA_BRANCH_STREAM
cd $R
DB=$(ls gpurun_out/s_trace/*/run_results.db gpurun_out/s_trace/run_results.db 2>/dev/null | head -1)
python3 tools/shape_trace.py $DB gpurun_out/s_trace.err > gpurun_out/r04_shape_trace.txt 2>&1
echo done
