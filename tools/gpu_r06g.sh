# Round 6: default bench line (with the live replay trace), pool sizes 8 / 16 / 32, and the flash
# threshold for P = 8 (DFCSA_LSA_FLASH_MIN_N=32 puts its 64 tokens on the flash kernels)
mkdir -p gpurun_out
T=${TAG:-r06g}
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err || exit 1
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace --steps 30 --warmup 5"
: > gpurun_out/${T}_pools.jsonl
for p in 4 8 16 32; do
  timeout -k 10 300 python bench.py --pool $p $S >> gpurun_out/${T}_pools.jsonl 2>> gpurun_out/${T}_pools.err || exit 1
done
DFCSA_LSA_FLASH_MIN_N=32 timeout -k 10 300 python bench.py --pool 8 $S >> gpurun_out/${T}_pools.jsonl 2>> gpurun_out/${T}_pools.err || exit 1
DFCSA_LSA_FLASH_MIN_N=8 timeout -k 10 300 python bench.py --pool 4 $S >> gpurun_out/${T}_pools.jsonl 2>> gpurun_out/${T}_pools.err || exit 1
python -c "
import json
for l in open('gpurun_out/${T}_pools.jsonl'):
    d = json.loads(l); print(d['config']['pool_size'], d['value'], d['ms_per_step'])
"
