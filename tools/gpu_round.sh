# one GPU call: tests, bench, per-call GEMM breakdown
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b.log 2>&1
timeout -k 10 200 python tools/step_breakdown.py > gpurun_out/sb.log 2>&1
