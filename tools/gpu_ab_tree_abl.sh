# Same-box A/B of the working tree against the snapshot in abl/tree/ (an earlier commit's bench.py,
# package and libdfcsa.so): 3 alternating rounds of the default bench, 150 timed steps each.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-kernel-timing --steps 150 --warmup 10"
for rep in 1 2 3; do
  (cd abl/tree && timeout -k 10 300 python bench.py $B > ../../gpurun_out/abl_old_$rep.json 2> ../../gpurun_out/abl_old_$rep.err) || { echo "old failed"; exit 1; }
  timeout -k 10 300 python bench.py $B > gpurun_out/abl_new_$rep.json 2> gpurun_out/abl_new_$rep.err || { echo "new failed"; exit 1; }
  python3 -c "import json;a=json.load(open('gpurun_out/abl_old_$rep.json'));b=json.load(open('gpurun_out/abl_new_$rep.json'));print('old', a['value'], 'new', b['value'])"
done
