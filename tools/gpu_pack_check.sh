mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "model or cfg2 or parity2 or zoo or transunet or unet or pack or block or fra_unet" > gpurun_out/pack_tests.log 2>&1 || { tail -30 gpurun_out/pack_tests.log; exit 1; }
tail -1 gpurun_out/pack_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/pack_bench.json 2>/dev/null
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/p_pack
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/p_pack -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-val-dice --no-trainer-faithful > $R/gpurun_out/p_pack.log 2>&1
