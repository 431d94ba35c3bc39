# Round-2 final evidence: all GPU tests, smoke, default bench, kernel trace, FETCH/WRITE + SQ passes
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/gpu_tests.log
set -e
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/p_trace $R/gpurun_out/p_fetch $R/gpurun_out/p_write $R/gpurun_out/p_sq
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-val-dice --no-trainer-faithful > $R/gpurun_out/p_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/p_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-graph --no-val-dice --no-trainer-faithful > $R/gpurun_out/p_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/p_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-graph --no-val-dice --no-trainer-faithful > $R/gpurun_out/p_write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/p_sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-graph --no-val-dice --no-trainer-faithful > $R/gpurun_out/p_sq.log 2>&1
echo done
