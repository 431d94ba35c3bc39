# Round 6: kernel traces of the P = 32 step and of config 5 (full-resolution attention, 512^2) on the
# current build, for the per-kernel breakdown (tools/kt_top.py)
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace"
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_p32b $R/gpurun_out/kt_cfg5
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_p32b -o run -- python3 $R/bench.py --pool 32 --steps 10 --warmup 3 --no-kernel-timing $S > $R/gpurun_out/kt_p32b.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_cfg5 -o run -- python3 $R/bench.py --model fullres --img 512 --batch 2 --steps 3 --warmup 1 --no-kernel-timing $S > $R/gpurun_out/kt_cfg5.log 2>&1 || exit 1
echo done
