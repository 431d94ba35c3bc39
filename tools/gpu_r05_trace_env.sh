# Kernel traces of the replayed default step under two environment settings, same box:
#   ENV_A / ENV_B (e.g. "DFCSA_RES_SCALE_SIDE=0") -> gpurun_out/kt_envA, kt_envB
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_envA $R/gpurun_out/kt_envB
S="--steps 10 --warmup 3 --no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing"
env $ENV_A timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_envA -o run -- python3 $R/bench.py $S > $R/gpurun_out/kt_envA.log 2>&1 || exit 1
env $ENV_B timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_envB -o run -- python3 $R/bench.py $S > $R/gpurun_out/kt_envB.log 2>&1 || exit 1
tail -1 $R/gpurun_out/kt_envA.log; tail -1 $R/gpurun_out/kt_envB.log
