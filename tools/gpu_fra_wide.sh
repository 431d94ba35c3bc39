# Wide-layer FRA backward (value-chunked MFMA kernels): parity tests, then config-5 bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fra_unet.py tests/test_gpu_fra_longn.py -x -v --timeout 200 --timeout-method thread > gpurun_out/fra_wide_tests.log 2>&1
timeout -k 10 240 python bench.py --model fullres --img 512 --batch 2 --steps 4 --warmup 2 --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/bench_fullres_r02.json 2> gpurun_out/bench_fullres_r02.err
