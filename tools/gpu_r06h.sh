# Round 6: is the GEMM path's saved forward state different in value or in identity? (P = 16, B = 2)
mkdir -p gpurun_out
: > gpurun_out/r06h_diag.log
for v in "USE_F=bmm USE_B=row STRIDES=1" "USE_F=bmm USE_B=row COPY=1" "USE_F=row USE_B=row COPY=2"; do
  echo "== $v" >> gpurun_out/r06h_diag.log
  env $v timeout -k 10 150 python -u tools/lsa_bmm_diag.py >> gpurun_out/r06h_diag.log 2>&1 || { rc=$?; echo "diag rc=$rc" >> gpurun_out/r06h_diag.log; exit $rc; }
done
bash tools/gpu_r06g.sh
