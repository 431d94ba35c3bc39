set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/p_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful > $R/gpurun_out/p_trace.log 2>&1
cd $R && python3 tools/rocpd_export.py stats $(find gpurun_out/p_trace -name '*.db' | head -1) gpurun_out/p_trace_stats.csv
python3 tools/trace_gaps.py $(find gpurun_out/p_trace -name '*.db' | head -1) > gpurun_out/gaps.log
