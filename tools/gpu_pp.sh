set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 200 python tools/pp_check.py 0,22,25 > gpurun_out/pp.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
