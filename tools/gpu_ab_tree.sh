# Same-box A/B of the working tree against the snapshot in _ab_base/ (built from an earlier
# commit): alternating default bench runs, 3 each.  Extra env: $AB_BASE_ENV (base runs), $AB_NEW_ENV (working tree).
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
for i in 1 2 3; do
(cd _ab_base && env $AB_BASE_ENV timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > ../gpurun_out/ab_base_$i.json 2> ../gpurun_out/ab_base_$i.err)
env $AB_NEW_ENV timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/ab_new_$i.json 2> gpurun_out/ab_new_$i.err
done
