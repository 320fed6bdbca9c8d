# round 6: bf16 tap-reuse weight-gradient split cap (PSX_AB_W3CAP) step A/B
set -o pipefail
mkdir -p gpurun_out
for c in 128 512; do
  bash scripts/prof/r6_ab.sh "PSX_AB_W3CAP=256" "PSX_AB_W3CAP=$c" --dtype bf16 --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/w3cap_bf16_$c.jsonl
done
bash scripts/prof/r6_ab.sh "PSX_AB_W3CAP=256" "PSX_AB_W3CAP=128" --model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/w3cap_r50_128.jsonl
