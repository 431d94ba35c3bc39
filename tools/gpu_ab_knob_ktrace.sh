# Per-kernel A/B of one tuning knob on the default bench step: kernel traces with DFCSA_TUNE=$1
# (arm B) and without (arm A), same box; compare with python tools/kt_compare.py
# gpurun_out/kt_A/*/run_results.db gpurun_out/kt_B/*/run_results.db
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_A $R/gpurun_out/kt_B
B="--steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_A -o run -- python3 $R/bench.py $B > $R/gpurun_out/kt_A.log 2>&1 || exit 1
DFCSA_TUNE=$1 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_B -o run -- python3 $R/bench.py $B > $R/gpurun_out/kt_B.log 2>&1 || exit 1
tail -1 $R/gpurun_out/kt_A.log; tail -1 $R/gpurun_out/kt_B.log
