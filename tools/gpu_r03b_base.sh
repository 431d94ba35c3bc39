# Session baseline on a fresh box: bench line (no CPU leg), kernel trace of the step, per-launch table.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful"
timeout -k 10 300 python bench.py $B > gpurun_out/bench_base.json 2> gpurun_out/bench_base.err || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/p_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_trace -o run -- python3 $R/bench.py --steps 4 --warmup 2 --no-graph --no-kernel-timing $B > $R/gpurun_out/p_trace.log 2>&1 || exit 1
cd $R
DB=$(ls gpurun_out/p_trace/*/run_results.db gpurun_out/p_trace/run_results.db 2>/dev/null | head -1)
python3 tools/step_kernels.py $DB 80 > gpurun_out/step_kernels.txt 2>&1
echo done
