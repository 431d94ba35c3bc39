# Round-6 evidence on the current build (gpurun_out/$TAG*): default bench line, smoke, the secondary
# BASELINE configs (1, 3 P=8, 4 fp32 + bf16, 5), kernel trace + stats, FETCH / WRITE passes and one
# SQ pass of the bench step.  TAG defaults to r06.  The kernel trace runs the timed replays only
# (--no-kernel-timing) so `rocpd_export.py replay` isolates the replayed step.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
T=${TAG:-r06}
cd $R
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace"
: > gpurun_out/${T}_bench_secondary.jsonl
for args in "--model unet --img 64 --batch 2 --precision fp32 --steps 50 --warmup 10" \
            "--pool 8 --steps 20 --warmup 5" \
            "--pool 16 --steps 20 --warmup 5" \
            "--pool 32 --steps 20 --warmup 5" \
            "--model transunet --batch 8 --precision fp32 --steps 10 --warmup 3" \
            "--model transunet --batch 8 --precision bf16 --steps 10 --warmup 3" \
            "--model fullres --img 512 --batch 2 --steps 4 --warmup 2"; do
  timeout -k 10 400 python bench.py $args $S >> gpurun_out/${T}_bench_secondary.jsonl 2>> gpurun_out/${T}_bench_secondary.err || exit 1
done
echo part1 done
