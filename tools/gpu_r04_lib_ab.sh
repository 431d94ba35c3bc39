# Same-box A/B of the working-tree libdfcsa.so against a snapshot library (arm A: DFCSA_LIB=$1):
# GPU tests of the touched kernels ($2 = pytest -k expression), per-kernel traces, 3 step rounds.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
BASE=$1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_fused_ref.py -k "$2" > gpurun_out/lab_tests.log 2>&1 || { tail -30 gpurun_out/lab_tests.log; exit 1; }
tail -1 gpurun_out/lab_tests.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_A $R/gpurun_out/kt_B
B="--steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing"
DFCSA_LIB=$R/$BASE timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_A -o run -- python3 $R/bench.py $B > $R/gpurun_out/kt_A.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_B -o run -- python3 $R/bench.py $B > $R/gpurun_out/kt_B.log 2>&1 || exit 1
cd $R
python3 tools/kt_compare.py $(ls gpurun_out/kt_A/*/run_results.db gpurun_out/kt_A/run_results.db 2>/dev/null | head -1) \
  $(ls gpurun_out/kt_B/*/run_results.db gpurun_out/kt_B/run_results.db 2>/dev/null | head -1) 25 > gpurun_out/lab_ktc.txt 2>&1
bash tools/gpu_ab_envs.sh "base:DFCSA_LIB=$R/$BASE" "new:DFCSA_X=0"
