# Profiles of the bench command committed under profiles/ (kernel trace + stats, PMC passes)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_bench $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-val-dice > $R/gpurun_out/prof_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-val-dice --no-kernel-timing --no-graph > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-val-dice --no-kernel-timing --no-graph > $R/gpurun_out/pmc_write.log 2>&1
