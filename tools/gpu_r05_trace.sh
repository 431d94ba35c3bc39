# Kernel trace of the default bench step (graph replay): gpurun_out/kt_cur/*.db for tools/kt_*.py.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_cur
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_cur -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing > $R/gpurun_out/kt_cur.log 2>&1 || exit 1
tail -1 $R/gpurun_out/kt_cur.log
find $R/gpurun_out/kt_cur -name "*.db" | head
