set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fra_unet.py -q --timeout 200 --timeout-method thread -k "fullres_model_fp32 or unet_matches" > gpurun_out/fra_fix.log 2>&1 || echo "fra tests failed" >> gpurun_out/fra_fix.log
timeout -k 10 200 python tools/step_breakdown.py > gpurun_out/sb.log 2>&1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_cur
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cur -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-graph > $R/gpurun_out/prof_cur.log 2>&1
