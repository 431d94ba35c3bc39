# One bench line per ablation-zoo model (224^2, B=16 per GPU, P=8 as in configs/config_ablation*.yaml)
set -e
mkdir -p gpurun_out
: > gpurun_out/zoo_bench.jsonl
for m in baseline attn_only addition concat encoder_only decoder_only both_standard; do
  timeout -k 10 200 python bench.py --model $m --pool 8 --steps 10 --warmup 3 --no-cpu-baseline --no-val-dice >> gpurun_out/zoo_bench.jsonl 2>> gpurun_out/zoo_bench.err
done
