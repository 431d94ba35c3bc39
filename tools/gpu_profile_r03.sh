# Round-3 evidence on the current build: default bench line, kernel trace + stats, FETCH / WRITE
# passes and one SQ pass of the bench step (profiles/r03*), smoke.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/p_trace $R/gpurun_out/p_fetch $R/gpurun_out/p_write $R/gpurun_out/p_sq
B="--no-cpu-baseline --no-val-dice --no-trainer-faithful"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 $B > $R/gpurun_out/p_trace.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/p_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-kernel-timing --no-graph $B > $R/gpurun_out/p_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/p_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-kernel-timing --no-graph $B > $R/gpurun_out/p_write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/p_sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-kernel-timing --no-graph $B > $R/gpurun_out/p_sq.log 2>&1 || exit 1
echo profile done
