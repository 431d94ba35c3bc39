set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "large_tiles or streaming" > gpurun_out/t.log 2>&1
timeout -k 10 300 python tools/gemm_bench.py 14,15,17,18 > gpurun_out/gb.log 2>&1
timeout -k 10 300 python tools/stream_bench.py > gpurun_out/sbench.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b.log 2>&1
timeout -k 10 200 python tools/step_breakdown.py > gpurun_out/sb.log 2>&1
