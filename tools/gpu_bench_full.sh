# The default bench line (CPU baseline, val Dice, Trainer-faithful leg) and the P=8 (config 3) per-GPU line.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
timeout -k 10 200 python bench.py --pool 8 --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/bench_p8.json 2> gpurun_out/bench_p8.err
