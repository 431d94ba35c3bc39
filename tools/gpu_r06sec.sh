# Round 6: the secondary bench lines only (P = 8 / 16 / 32, TransUNet fp32 / bf16, config 5) on the
# current build -> gpurun_out/$TAG_bench_secondary.jsonl
mkdir -p gpurun_out
T=${TAG:-r06g}
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
echo secondary done
