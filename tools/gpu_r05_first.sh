# Round 5, first call: the timed-config (B = 16) parity test, the default bench line and the DDP
# code path (world-1 RCCL group, bucket reducer) at the headline geometry, same box.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
T=${TAG:-r05a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity2.py -k "timed_config or cfg2_geometry_bf16_train" -v -s --timeout 240 --timeout-method thread > gpurun_out/${T}_b16_test.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_b16_test.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing --steps 100 --warmup 10"
for i in 1 2; do
timeout -k 10 200 python bench.py $S >> gpurun_out/${T}_bench_plain.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
timeout -k 10 200 python bench.py $S --ddp-rehearsal >> gpurun_out/${T}_bench_ddp.jsonl 2>> gpurun_out/${T}_bench.err || exit 1
done
cat gpurun_out/${T}_bench_plain.jsonl gpurun_out/${T}_bench_ddp.jsonl | python -c "import sys,json; [print(json.loads(l)['value'], json.loads(l)['config']['ddp_path']) for l in sys.stdin]"
exit $rc
