# kernel trace of the default bench command (no PMC passes)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-val-dice > $R/gpurun_out/prof_bench.log 2>&1
