# Verify HEAD on a fresh box: the RCCL graph rehearsal standalone (full log), then the GPU tests,
# smoke(), the default bench line and a kernel trace of the bench command.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
MASTER_ADDR=127.0.0.1 timeout -k 10 240 python -u tools/rccl_graph_check.py > gpurun_out/rccl_check.log 2>&1
echo "rccl rc=$?"
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity2.py::test_rccl_bucket_reducer_graph_replay_equals_eager > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/p_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful > $R/gpurun_out/p_trace.log 2>&1
