# Secondary BASELINE configs on the current build (one JSON line each): config 1 UNet 64^2 fp32 B=2;
# config 3 P=8 224^2 bf16 B=16 per GPU; config 4 TransUNet 224^2 fp32 and bf16 B=8; config 5 FRA 512^2 bf16 B=2
set -e
mkdir -p gpurun_out
: > gpurun_out/secondary.jsonl
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful"
timeout -k 10 200 python bench.py --model unet --img 64 --batch 2 --precision fp32 --steps 50 --warmup 10 $B >> gpurun_out/secondary.jsonl
timeout -k 10 200 python bench.py --pool 8 $B >> gpurun_out/secondary.jsonl
timeout -k 10 200 python bench.py --model transunet --img 224 --batch 8 --precision fp32 --steps 10 --warmup 3 $B >> gpurun_out/secondary.jsonl
timeout -k 10 200 python bench.py --model transunet --img 224 --batch 8 --precision bf16 --steps 10 --warmup 3 $B >> gpurun_out/secondary.jsonl
timeout -k 10 240 python bench.py --model fullres --img 512 --batch 2 --steps 4 --warmup 2 $B >> gpurun_out/secondary.jsonl
