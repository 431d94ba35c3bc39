# Config 4 (TransUNet bf16, B = 8) bench line and kernel trace (gpurun_out/tu_trace/*.db).
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
S="--model transunet --batch 8 --precision bf16 --no-cpu-baseline --no-val-dice --no-trainer-faithful"
cd $R
timeout -k 10 300 python bench.py $S --steps 10 --warmup 3 > gpurun_out/tu_bench.json 2> gpurun_out/tu_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/tu_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tu_trace -o run -- python3 $R/bench.py $S --steps 10 --warmup 3 --no-kernel-timing > $R/gpurun_out/tu_trace.log 2>&1 || exit 1
find $R/gpurun_out/tu_trace -name "*.db" -o -name "*stats.csv" | head
