mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python3 tools/wgrad_bench.py "base:" "nst3:14=3" "nst4:14=4" "n64_3:24=3" "n64_4:24=4" "t1024:2=1024" "t256:2=256" "wide18:18=1" "narrow0:8=0" "big1:17=1" "big2:17=2" "big3:17=3" > gpurun_out/wgb.jsonl 2> gpurun_out/wgb.err
echo rc=$?
