# Round 6: same-box A/B of the large-pool LSA variants (P = 16 / 32): dgamma as a separate sum (default)
# vs in-kernel, pool windows batched per workgroup (knob 45) vs not; then a P = 32 kernel trace
mkdir -p gpurun_out
T=${TAG:-r06o}
R=$GRAFT_REPO_ROOT
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 40 --warmup 5"
: > gpurun_out/${T}_ab.txt
for round in 1 2; do
  for v in "X=0" "DFCSA_LSA_DGAMMA_SPLIT=0" "DFCSA_TUNE=45=1"; do
    for p in 16 32; do
      out=$(env $v timeout -k 10 300 python bench.py --pool $p $S 2>> gpurun_out/${T}_ab.err) || exit 1
      echo "$round $v P=$p $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/${T}_ab.txt
    done
  done
done
cat gpurun_out/${T}_ab.txt
cd /tmp && export TMPDIR=/tmp
S2="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing --no-live-trace --steps 10 --warmup 3"
rm -rf $R/gpurun_out/kt_p32
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt_p32 -o run -- python3 $R/bench.py --pool 32 $S2 > $R/gpurun_out/kt_p32.log 2>&1 || exit 1
