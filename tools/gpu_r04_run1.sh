# Round-4 check: the changed/new GPU tests, then a same-box A/B of the cooperative split-K wgrad
# reduction (knob 31) on the default bench.  Test failures (rc 1) do not stop the bench; any other
# non-zero status (timeout, abort, fault) ends the script.
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity2.py tests/test_gpu_trainer.py tests/test_gpu_kernels.py "tests/test_gpu_fra_unet.py::test_fullres_model_512_bf16_train_step_factory" -s > gpurun_out/r04_t1.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="--no-val-dice --no-cpu-baseline --no-trainer-faithful --steps 30 --warmup 5"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/r04_ab_coop_$i.json 2> gpurun_out/r04_ab_coop_$i.err || exit 1
  DFCSA_TUNE=31=0 timeout -k 10 300 python bench.py $B > gpurun_out/r04_ab_nocoop_$i.json 2> gpurun_out/r04_ab_nocoop_$i.err || exit 1
done
grep -h -o '"value": [0-9.]*' gpurun_out/r04_ab_*.json
