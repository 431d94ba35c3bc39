# Same-box A/B of the working tree against the snapshot in _ab_prev/ (an earlier commit's bench.py,
# package and libdfcsa.so): 3 alternating rounds of the default bench, 150 timed steps each.
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing --steps 150 --warmup 10"
for rep in 1 2 3; do
  (cd _ab_prev && timeout -k 10 300 python bench.py $B > ../gpurun_out/ab_prev_$rep.json 2> ../gpurun_out/ab_prev_$rep.err) || { echo "prev failed"; exit 1; }
  env $AB_NEW_ENV timeout -k 10 300 python bench.py $B > gpurun_out/ab_new_$rep.json 2> gpurun_out/ab_new_$rep.err || { echo "new failed"; exit 1; }
  python3 -c "import json;a=json.load(open('gpurun_out/ab_prev_$rep.json'));b=json.load(open('gpurun_out/ab_new_$rep.json'));print('prev', a['value'], 'new', b['value'])"
done
