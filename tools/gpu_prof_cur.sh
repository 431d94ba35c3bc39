set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_cur
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cur -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-graph --no-val-dice > $R/gpurun_out/prof_cur.log 2>&1
