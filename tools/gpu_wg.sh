set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "wgrad" > gpurun_out/t.log 2>&1
timeout -k 10 300 python tools/wgrad_bench.py > gpurun_out/wb.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b.log 2>&1
