# Round 3: buffer-descriptor LDS-DMA in the conv tile kernels -- kernel tests, per-layer timing, bench.
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
step ktests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fused_ref.py tests/test_gpu_val_parity.py -q -x --timeout 240 --timeout-method thread
step layers 300 python -u tools/halo_bench.py fwd,dgrad
step bench 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful --steps 30
echo done
