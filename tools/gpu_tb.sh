# GPU tests + two default bench lines (no CPU baseline / val / trainer legs)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/tb_1.json 2> gpurun_out/tb_1.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/tb_2.json 2> gpurun_out/tb_2.err
