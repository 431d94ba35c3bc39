# Env A/B on the current defaults: input gradient before the side-stream weight gradients, the split
# block-input gradient, and no branch stream.
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_envs.sh "base:X=0" "dxfirst:DFCSA_DX_FIRST=1" "split:DFCSA_SPLIT_DX=1" "early:DFCSA_WGRAD_LATE=0"
