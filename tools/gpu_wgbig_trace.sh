mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/wgt
WGRAD_MODES=default,big1,big2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wgt -o run -- python3 $R/tools/wgrad_shapes.py > $R/gpurun_out/wgt.log 2>&1
