# Round 5, TransUNet: the config-4 tests (fixtures, bf16 autocast bar, kernels) and the bf16 / fp32
# bench lines on the current build.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
T=${TAG:-tu2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_transunet.py tests/test_gpu_model.py -k "transunet or TransUNet or groupnorm or colsum or unet" -q -x --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
S="--model transunet --batch 8 --no-cpu-baseline --no-val-dice --no-trainer-faithful"
timeout -k 10 300 python bench.py $S --precision bf16 --steps 20 --warmup 5 > gpurun_out/${T}_bench.jsonl 2> gpurun_out/${T}_bench.err || exit 1
timeout -k 10 300 python bench.py $S --precision fp32 --steps 10 --warmup 3 >> gpurun_out/${T}_bench.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
python -c "
import json
for l in open('gpurun_out/${T}_bench.jsonl'): d=json.loads(l); print(d['dtype'], d['value'], d['ms_per_step'])"
