# Round 6: kernel traces of the P = 16 / 32 bench steps (timed replays only), per-kernel stats
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing --no-live-trace --steps 10 --warmup 3"
for p in 32 16; do
  rm -rf $R/gpurun_out/kt_p$p
  ${ENVV} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_p$p -o run -- python3 $R/bench.py --pool $p $S > $R/gpurun_out/kt_p$p.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/kt_p$p.log
done
