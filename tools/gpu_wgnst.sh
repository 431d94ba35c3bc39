set -e
mkdir -p gpurun_out
WGRAD_MODES=default,nst3,nst4,nst3_t256,nst4_t256,t1024 timeout -k 10 300 python tools/wgrad_shapes.py > gpurun_out/wgnst.log 2>&1
