# Quick GPU check: the given test files (TESTS env), then a short default bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_model.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/check_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err
