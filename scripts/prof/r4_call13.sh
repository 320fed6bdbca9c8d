set -o pipefail
for p in 0 4 8 16 24; do PSX_SK_PROBE=$p BN=128 timeout -k 10 60 python scripts/prof/sk_probe.py || exit 1; done
