# Round 3: halo-tile conv variants (knob 22) -- correctness and per-layer timing.
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
step halo_tests_v0 300 python -u -m pytest tests/test_gpu_halo.py -q -x --timeout 120 --timeout-method thread
step halo_tests_v1 300 env DFCSA_TUNE=22=1 python -u -m pytest tests/test_gpu_halo.py -q -x --timeout 120 --timeout-method thread
step halo_layers_v0 300 python -u tools/halo_bench.py fwd,dgrad
step halo_layers_v1 300 env DFCSA_TUNE=22=1 python -u tools/halo_bench.py fwd,dgrad

GEMM_SHAPES="3x3" timeout -k 10 400 python -u tools/gemm_bench.py 0,17,11,14,16,10,18,13 > gpurun_out/gemm_cfgs_r03.jsonl 2>&1; echo "gemm_cfgs rc=$?"
bash tools/gpu_r03_pmc_wgrad.sh || exit 1
echo done2
