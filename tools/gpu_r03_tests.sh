# Round-3 check on a fresh box: the whole -m gpu suite (new: fused kernels vs torch, slab
# canaries/capacity, bf16 config-2 backward vs the reference's autocast, Trainer replay / DP),
# then smoke() and the default bench line.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 240 --timeout-method thread -x > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
