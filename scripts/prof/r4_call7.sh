set -o pipefail
mkdir -p gpurun_out
AB_CFGS="_ PSX_WG_SHARE=0.5 PSX_WG_SHARE=0.75 PSX_TAIL_SPLIT=0 PSX_WINO_WGF_Q=16 PSX_WINO_BWDFOLD=0" bash scripts/prof/ab_env.sh || exit 1
