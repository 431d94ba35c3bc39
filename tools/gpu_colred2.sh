set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_colred.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/colred.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err
bash tools/gpu_trace.sh
