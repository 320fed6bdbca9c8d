set -o pipefail
mkdir -p gpurun_out
bash scripts/prof/r6_ab.sh "PSX_AB_W3CAP=128" "PSX_AB_W3CAP=64" --dtype bf16 --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/w3cap_bf16_128v64.jsonl
bash scripts/prof/r6_ab.sh "PSX_AB_W3CAP=256" "PSX_AB_W3CAP=128" --dtype bf16 --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/w3cap_bf16_256v128b.jsonl
