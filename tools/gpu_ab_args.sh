# A/B of bench.py argument sets on the default bench (same box, 3 rounds): gpu_ab_args.sh "<label>:<args>" ...
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing --steps 150 --warmup 10"
for rep in 1 2 3; do
  for arm in "$@"; do
    lab=${arm%%:*}; args=${arm#*:}
    timeout -k 10 300 python bench.py $B $args > gpurun_out/aba_${lab}_$rep.json 2> gpurun_out/aba_${lab}_$rep.err || { echo "bench $lab failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/aba_${lab}_$rep.json'));print('$lab', $rep, d['value'], d['ms_per_step'], d['launch'])"
  done
done
