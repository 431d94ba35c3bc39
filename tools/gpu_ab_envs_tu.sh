# Same-box A/B of environment settings on the TransUNet bf16 bench (config 4): three alternating
# rounds.  usage: bash tools/gpu_ab_envs_tu.sh "label:VAR=v VAR2=v" ...
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-tu_ab}.txt
: > $OUT
S="--model transunet --batch 8 --precision bf16 --no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing --steps 30 --warmup 5"
for r in 1 2 3; do
  for arm in "$@"; do
    lab=${arm%%:*}; envs=${arm#*:}
    v=$(env $envs timeout -k 10 200 python bench.py $S 2>/dev/null | python -c "import sys,json; print(json.loads(sys.stdin.read())['value'])") || exit 1
    echo "$r $lab $v" | tee -a $OUT
  done
done
