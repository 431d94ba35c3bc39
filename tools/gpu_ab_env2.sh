# GPU tests named by $TESTS (pytest -k expression over tests/ -m gpu), then a same-box A/B of the
# default bench under env $AB_A vs $AB_B (alternating, $AB_N runs each).
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$TESTS" > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -2 gpurun_out/ab_tests.log
fi
for i in $(seq 1 ${AB_N:-2}); do
  env $AB_A timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/ab_a_$i.json 2> gpurun_out/ab_a_$i.err || exit 1
  env $AB_B timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/ab_b_$i.json 2> gpurun_out/ab_b_$i.err || exit 1
done
python - <<'PY'
import json, glob
for k in ("a", "b"):
    v = [json.loads(open(f).read().strip().splitlines()[-1])["value"] for f in sorted(glob.glob(f"gpurun_out/ab_{k}_*.json"))]
    print(k, v)
PY
