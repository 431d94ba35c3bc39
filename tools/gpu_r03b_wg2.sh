mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
WG_SHAPES=3x3 timeout -k 10 500 python3 tools/wgrad_bench.py "warm:" "base:" "halo:20=1" "halo_t1024:20=1;2=1024" "base2:" > gpurun_out/wgb2.jsonl 2> gpurun_out/wgb2.err
echo rc=$?
