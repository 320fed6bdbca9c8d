set -o pipefail
AB_CFGS="_ PSX_FORCE_DIST=0" bash scripts/prof/ab_env.sh || exit 1
