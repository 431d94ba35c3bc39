# A/B of the headline bench: _oldtree (a committed baseline build) vs the current tree, alternated
# twice in one box session (box-to-box variation is ~1 %).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
: > $R/gpurun_out/ab.jsonl
for i in 1 2; do
  cd $R/_oldtree && timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful > $R/gpurun_out/ab_o.json 2>/dev/null
  echo "{\"tree\": \"old\", \"line\": $(cat $R/gpurun_out/ab_o.json)}" >> $R/gpurun_out/ab.jsonl
  cd $R && timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful > $R/gpurun_out/ab_n.json 2>/dev/null
  echo "{\"tree\": \"new\", \"line\": $(cat $R/gpurun_out/ab_n.json)}" >> $R/gpurun_out/ab.jsonl
done
