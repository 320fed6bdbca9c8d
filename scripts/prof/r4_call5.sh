set -o pipefail
mkdir -p gpurun_out
AB_CFGS="PSX_WINO_WGF=0 PSX_WINO_WGF=1 PSX_WINO_WGF_MINHW=16" bash scripts/prof/ab_env.sh || exit 1
bash scripts/prof/step_prof.sh
