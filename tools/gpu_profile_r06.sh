# Round-6 evidence on the current build (gpurun_out/$TAG*): default bench line, smoke, the secondary
# BASELINE configs (1, 3 P=8, 4 fp32 + bf16, 5), kernel trace + stats, FETCH / WRITE passes and one
# SQ pass of the bench step.  TAG defaults to r06.  The kernel trace runs the timed replays only
# (--no-kernel-timing) so `rocpd_export.py replay` isolates the replayed step.
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
T=${TAG:-r06}
cd $R
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
S="--no-cpu-baseline --no-val-dice --no-trainer-faithful --no-live-trace"
: > gpurun_out/${T}_bench_secondary.jsonl
for args in "--model unet --img 64 --batch 2 --precision fp32 --steps 50 --warmup 10" \
            "--pool 8 --steps 20 --warmup 5" \
            "--pool 16 --steps 20 --warmup 5" \
            "--pool 32 --steps 20 --warmup 5" \
            "--model transunet --batch 8 --precision fp32 --steps 10 --warmup 3" \
            "--model transunet --batch 8 --precision bf16 --steps 10 --warmup 3" \
            "--model fullres --img 512 --batch 2 --steps 4 --warmup 2"; do
  timeout -k 10 400 python bench.py $args $S >> gpurun_out/${T}_bench_secondary.jsonl 2>> gpurun_out/${T}_bench_secondary.err || exit 1
done
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
echo profile done
