set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_colred.py -x -v --timeout 120 --timeout-method thread > gpurun_out/colred.log 2>&1 || { tail -40 gpurun_out/colred.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity2.py -x -q -k cfg2_geometry_fp32 --timeout 200 --timeout-method thread > gpurun_out/cfg2.log 2>&1 || true
