mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$TESTS" > gpurun_out/ct_tests.log 2>&1 || { tail -30 gpurun_out/ct_tests.log; exit 1; }
tail -1 gpurun_out/ct_tests.log
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful 2>/dev/null | python -c "import json,sys; print('bench', json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])" || exit 1; done
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/p_ct
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/p_ct -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-val-dice --no-trainer-faithful > $R/gpurun_out/p_ct.log 2>&1
