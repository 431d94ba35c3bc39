# A/B of the branch stream (DFCSA_BRANCH_STREAM) on the headline bench, then the GPU tests
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
for i in 1 2; do
DFCSA_BRANCH_STREAM=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/ab_off_$i.json 2> gpurun_out/ab_off_$i.err
DFCSA_BRANCH_STREAM=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/ab_on_$i.json 2> gpurun_out/ab_on_$i.err
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
