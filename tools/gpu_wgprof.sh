set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/wgprof
WGRAD_MODES=unfused timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wgprof -o run -- python3 $R/tools/wgrad_shapes.py > $R/gpurun_out/wgprof.log 2>&1
find $R/gpurun_out/wgprof -name "*.db" -o -name "*stats*" | head
