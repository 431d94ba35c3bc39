mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py tests/test_gpu_zoo.py -k "block or lsa or model or attn or local or zoo" -x -q -rs --timeout 200 --timeout-method thread > gpurun_out/pool_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pool_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_ab_tree.sh
for f in gpurun_out/ab_base_*.json gpurun_out/ab_new_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'])"; done
