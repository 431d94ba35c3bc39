# Round 6: kernel trace of the TransUNet bf16 step (config 4) on the current build (tools/kt_top.py)
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace"
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_tu
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_tu -o run -- python3 $R/bench.py --model transunet --batch 8 --precision bf16 --steps 8 --warmup 3 --no-kernel-timing $S > $R/gpurun_out/kt_tu.log 2>&1 || exit 1
echo done
