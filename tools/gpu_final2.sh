# Full verification after a kernel change: GPU tests, smoke(), default bench, config-5 bench,
# attention microbenchmark, and the kernel trace of the config-5 bench.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
timeout -k 10 200 python bench.py --model fullres --img 512 --batch 2 --steps 4 --warmup 2 > gpurun_out/bench_fullres.json 2> gpurun_out/bench_fullres.err
timeout -k 10 200 python tools/fra_bench.py 0,15 > gpurun_out/fra_bench.log 2>&1
FRA_C=128 FRA_HW=256 timeout -k 10 120 python tools/fra_bench.py 0,15 > gpurun_out/fra_bench128.log 2>&1
bash tools/gpu_fra_prof.sh
