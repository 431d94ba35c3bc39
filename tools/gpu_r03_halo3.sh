# Round 3: halo-tile conv v3 -- correctness, per-layer timing against the row tiles, counters, bench A/B.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
step() {  # step <name> <timeout> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step ktests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fused_ref.py tests/test_gpu_val_parity.py tests/test_gpu_model.py -q -x --timeout 240 --timeout-method thread
step halo_tests 300 python -u -m pytest tests/test_gpu_halo.py -q -x --timeout 120 --timeout-method thread
step halo_layers 400 python -u tools/halo_bench.py fwd,dgrad,wgrad
B="python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful --steps 30"
step bench_nohalo 300 $B
step bench_halo 300 env DFCSA_TUNE=19=32768 $B
bash tools/gpu_r03_pmc_halo.sh || exit 1
echo done
