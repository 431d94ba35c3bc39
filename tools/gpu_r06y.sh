# Round 6: kernel traces of the P = 8 and P = 16 steps on the current build (tools/kt_top.py)
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace"
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_p8 $R/gpurun_out/kt_p16b
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_p8 -o run -- python3 $R/bench.py --pool 8 --steps 10 --warmup 3 --no-kernel-timing $S > $R/gpurun_out/kt_p8.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_p16b -o run -- python3 $R/bench.py --pool 16 --steps 10 --warmup 3 --no-kernel-timing $S > $R/gpurun_out/kt_p16b.log 2>&1 || exit 1
echo done
