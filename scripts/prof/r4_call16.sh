set -o pipefail
AB_CFGS="_ PSX_WINO_FUSED=1 PSX_WINO_FUSED=2 PSX_WINO_SK=1" bash scripts/prof/ab_env.sh || exit 1
