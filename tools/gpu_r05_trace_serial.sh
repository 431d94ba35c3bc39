# Kernel traces of the replayed default step with the side / branch streams serialised (kt_ser) and
# concurrent (kt_con), same box: per-kernel durations with and without co-running streams.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_ser $R/gpurun_out/kt_con
S="--steps 10 --warmup 3 --no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing"
DFCSA_SIDE_STREAM=0 DFCSA_BRANCH_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_ser -o run -- python3 $R/bench.py $S > $R/gpurun_out/kt_ser.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_con -o run -- python3 $R/bench.py $S > $R/gpurun_out/kt_con.log 2>&1 || exit 1
tail -1 $R/gpurun_out/kt_ser.log; tail -1 $R/gpurun_out/kt_con.log
