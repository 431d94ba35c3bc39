# config-4 bench line and its kernel trace
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python bench.py --model transunet --batch 8 --steps 10 --warmup 3 > gpurun_out/bench_transunet.json 2> gpurun_out/bench_transunet.err
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_tu
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_tu -o run -- python3 $R/bench.py --model transunet --batch 8 --steps 10 --warmup 3 --no-cpu-baseline --no-val-dice > $R/gpurun_out/prof_tu.log 2>&1
