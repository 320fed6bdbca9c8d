# round 6: fused Winograd weight-gradient workgroup target (PSX_AB_WFQ) step A/B, fp32
set -o pipefail
mkdir -p gpurun_out
for alt in "PSX_AB_WFQ=256" "PSX_AB_WFQ=1024"; do
  tag=${alt#PSX_AB_}
  bash scripts/prof/r6_ab.sh "PSX_X=0" "$alt" --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/wfq_fp32_$tag.jsonl
done
bash scripts/prof/r6_ab.sh "PSX_X=0" "PSX_AB_WFQ=256" --model resnet50 --codec topk --steps 10 --warmup 3 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wfq_r50_WFQ=256.jsonl
