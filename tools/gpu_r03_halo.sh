# halo kernels: correctness, then per-layer timing against the row-tile kernels
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -v -rs --timeout 120 --timeout-method thread > gpurun_out/halo_tests.log 2>&1
rc=$?; echo "halo_tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/halo_bench.py > gpurun_out/halo_bench.jsonl 2> gpurun_out/halo_bench.err
echo "halo_bench rc=$?"
