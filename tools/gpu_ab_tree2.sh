# Two alternating rounds of the default bench: _ab_base/ (an earlier commit) against the working tree.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful"
for i in 1 2; do
  (cd _ab_base && timeout -k 10 300 python bench.py $B > ../gpurun_out/ab_base_$i.json 2> ../gpurun_out/ab_base_$i.err) || exit 1
  timeout -k 10 300 python bench.py $B > gpurun_out/ab_new_$i.json 2> gpurun_out/ab_new_$i.err || exit 1
done
for f in gpurun_out/ab_base_*.json gpurun_out/ab_new_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['ms_per_step'])"; done
