set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/dev/fold_probe2.py || exit 1
Q="4,8,16,32,64" timeout -k 10 300 python bench/wino_wgrad_ab.py | tee gpurun_out/wgf_ab.jsonl || exit 1
bash scripts/prof/wgf_pmc.sh
