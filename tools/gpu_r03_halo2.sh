# halo conv v2: correctness, per-layer timing, the bf16 config-2 backward test
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -v -rs --timeout 120 --timeout-method thread > gpurun_out/halo_tests.log 2>&1
rc=$?; echo "halo_tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/halo_bench.py fwd,dgrad > gpurun_out/halo_bench2.jsonl 2> gpurun_out/halo_bench2.err
rc=$?; echo "halo_bench rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity2.py -v -s -rs --timeout 300 --timeout-method thread -k "cfg2_geometry_bf16_train" > gpurun_out/cfg2_bf16.log 2>&1
echo "cfg2_bf16 rc=$?"
