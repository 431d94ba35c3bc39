# Round-6 evidence, part 2: kernel traces (replayed step; class-timing pass), FETCH / WRITE / SQ passes,
# then the driver's -m gpu command line.  TAG defaults to r06.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
T=${TAG:-r06}
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace"
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/p_trace $R/gpurun_out/p_fetch $R/gpurun_out/p_write $R/gpurun_out/p_sq
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-kernel-timing $S > $R/gpurun_out/p_trace.log 2>&1 || exit 1
# the bench command with its class-timing pass: the last 20 steps of this trace are the serialised
# eager pass whose HIP-event class times the line reports (rocpd_export.py replay ... -> *_serial_classes.json)
rm -rf $R/gpurun_out/p_trace_timing
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_trace_timing -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-live-trace $S > $R/gpurun_out/p_trace_timing.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/p_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-kernel-timing --no-graph $S > $R/gpurun_out/p_fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/p_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-kernel-timing --no-graph $S > $R/gpurun_out/p_write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/p_sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-kernel-timing --no-graph $S > $R/gpurun_out/p_sq.log 2>&1 || exit 1
cd $R
timeout -k 10 900 python3 -m pytest tests/ -q -m gpu -p no:cacheprovider > gpurun_out/${T}_gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/${T}_gpu_suite.log; tail -3 gpurun_out/${T}_gpu_suite.log
exit $rc
