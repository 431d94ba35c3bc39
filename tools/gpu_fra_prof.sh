# kernel trace of the config-5 bench (full-resolution attention split fwd / dK,dV / dQ)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_fra
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fra -o run -- python3 $R/bench.py --model fullres --img 512 --batch 2 --steps 3 --warmup 1 --no-cpu-baseline --no-val-dice > $R/gpurun_out/prof_fra.log 2>&1
