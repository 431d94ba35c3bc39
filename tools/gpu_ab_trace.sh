# A/B kernel traces of the headline bench: the round-1 tree (_oldtree) and the current tree
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/ab_old $R/gpurun_out/ab_new
cd $R/_oldtree && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ab_old -o run -- python3 $R/_oldtree/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-val-dice --no-kernel-timing > $R/gpurun_out/ab_old.log 2>&1
cd $R && DFCSA_TUNE=12=-1 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ab_new -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-val-dice --no-kernel-timing --no-trainer-faithful > $R/gpurun_out/ab_new.log 2>&1
ls $R/gpurun_out/ab_old $R/gpurun_out/ab_new
