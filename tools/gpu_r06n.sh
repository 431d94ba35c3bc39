# Round 6: batched pooling windows -- LSA tests, P = 16 / 32 benches and kernel traces
mkdir -p gpurun_out
T=${TAG:-r06n}
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_lsa_flash.py "tests/test_gpu_model.py::test_lsa_fp32" "tests/test_gpu_kernels.py::test_lsa_up_bwd_rows_and_pool" tests/test_gpu_qk_ratio.py -q -p no:cacheprovider > gpurun_out/${T}_targeted.log 2>&1
rc=$?; echo "targeted rc=$rc" >> gpurun_out/${T}_targeted.log; tail -3 gpurun_out/${T}_targeted.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 30 --warmup 5"
: > gpurun_out/${T}_pools.jsonl
for p in 16 32; do
  timeout -k 10 300 python bench.py --pool $p $S >> gpurun_out/${T}_pools.jsonl 2>> gpurun_out/${T}_pools.err || exit 1
done
python -c "
import json
for l in open('gpurun_out/${T}_pools.jsonl'):
    d = json.loads(l); print(d['config']['pool_size'], d['value'], d['ms_per_step'])
"
cd /tmp && export TMPDIR=/tmp
S2="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing --no-live-trace --steps 10 --warmup 3"
for p in 32 16; do
  rm -rf $R/gpurun_out/kt_p$p
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_p$p -o run -- python3 $R/bench.py --pool $p $S2 > $R/gpurun_out/kt_p$p.log 2>&1 || exit 1
done
