# Pack-plan check: its GPU test, the per-kernel trace A/B against _ab_prev/ and one LDS counter
# pass (bank conflicts / LDS cycles) of the pack plan for both trees.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "pack or layout2 or lsa or dgrad1x1 or conv_transpose or relu_bn_pair" > gpurun_out/t_pack.log 2>&1 || { tail -30 gpurun_out/t_pack.log; exit 1; }
tail -1 gpurun_out/t_pack.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_fra_unet.py::test_unet_matches_reference tests/test_gpu_parity2.py -k "not rccl and not bench_ddp" > gpurun_out/t_pack2.log 2>&1 || { tail -30 gpurun_out/t_pack2.log; exit 1; }
tail -1 gpurun_out/t_pack2.log
tail -1 gpurun_out/t_pack.log
timeout -k 10 180 python tools/stream_minm_bench.py > gpurun_out/stream_minm.jsonl 2> gpurun_out/stream_minm.err || exit 1
cat gpurun_out/stream_minm.jsonl
AB_BASE=_ab_prev bash tools/gpu_ab_ktrace.sh || exit 1
cd /tmp && export TMPDIR=/tmp
B="--steps 2 --warmup 1 --no-kernel-timing --no-graph --no-cpu-baseline --no-val-dice --no-trainer-faithful"
rm -rf $R/gpurun_out/p_lds_new $R/gpurun_out/p_lds_prev
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $R/gpurun_out/p_lds_new -o run -- python3 $R/bench.py $B > $R/gpurun_out/p_lds_new.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $R/gpurun_out/p_lds_prev -o run -- python3 $R/_ab_prev/bench.py $B > $R/gpurun_out/p_lds_prev.log 2>&1 || exit 1
cd $R
for t in prev new; do echo "== $t"; python3 tools/pmc_summary.py pack_plan $(ls gpurun_out/p_lds_$t/*/run_results.db gpurun_out/p_lds_$t/run_results.db 2>/dev/null); done
cd $R && bash tools/gpu_ab_tree3.sh
