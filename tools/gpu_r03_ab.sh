# Round 3: the val-parity test, halo v2 counters and a wgrad in-kernel-reduction A/B on one box.
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
step valpar 300 python -u -m pytest tests/test_gpu_val_parity.py -v -s --timeout 240 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful --steps 30"
step ab_base 300 $B
step ab_fuse12 300 env DFCSA_TUNE=12=1 $B
step ab_fuse13 300 env DFCSA_TUNE=13=8 $B
bash tools/gpu_r03_pmc_halo.sh || exit 1
echo done
