# Per-kernel A/B: kernel trace of the default bench step for the build in _ab_base/ (an earlier
# commit, see gpu_ab_tree.sh) and for the working tree; compare with
# `python tools/rocpd_export.py stats` on gpurun_out/kt_{base,new}/*/run_results.db.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt_base $R/gpurun_out/kt_new
B="--steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_base -o run -- python3 $R/${AB_BASE:-_ab_base}/bench.py $B > $R/gpurun_out/kt_base.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_new -o run -- python3 $R/bench.py $B > $R/gpurun_out/kt_new.log 2>&1 || exit 1
tail -1 $R/gpurun_out/kt_base.log; tail -1 $R/gpurun_out/kt_new.log
