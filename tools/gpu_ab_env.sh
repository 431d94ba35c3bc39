# A/B an environment switch on the headline bench: bash tools/gpu_ab_env.sh VAR  (0 vs 1, twice)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
V=$1
for i in 1 2; do
env $V=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/ab_0_$i.json 2> gpurun_out/ab_0_$i.err
env $V=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/ab_1_$i.json 2> gpurun_out/ab_1_$i.err
done
