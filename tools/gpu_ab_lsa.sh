# LightSelfAttention kernel changes: their tests, then the per-kernel trace A/B and two rounds of
# the tree A/B (working tree against _ab_base/).
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py tests/test_gpu_zoo.py tests/test_gpu_parity2.py -k "block or lsa or model or attn or local or zoo or cfg2 or fra or pool or entry" -x -q -rs --timeout 200 --timeout-method thread > gpurun_out/lsa_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/lsa_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_ab_ktrace.sh || exit 1
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful"
for i in 1 2; do
  (cd _ab_base && timeout -k 10 300 python bench.py $B > ../gpurun_out/ab_base_$i.json 2> ../gpurun_out/ab_base_$i.err) || exit 1
  timeout -k 10 300 python bench.py $B > gpurun_out/ab_new_$i.json 2> gpurun_out/ab_new_$i.err || exit 1
done
for f in gpurun_out/ab_base_*.json gpurun_out/ab_new_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'])"; done
