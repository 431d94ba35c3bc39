set -e
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 300 python tools/gemm_bench.py 0 > gpurun_out/gb.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b.log 2>&1
