set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT; cd $R
for i in 1 2; do
for t in "17=0,18=0" "17=1,18=0" "17=0,18=1" "17=1,18=1"; do
DFCSA_TUNE=$t timeout -k 10 300 python bench.py --no-cpu-baseline --no-val-dice --no-trainer-faithful > gpurun_out/kn_${t}_$i.json 2> /dev/null
done
done
