# round 6: more grid heuristics, temporary knobs: Winograd weight-gradient q target (PSX_AB_WQT),
# weight-gradient reduction width target (PSX_AB_RCW), conv 64x128-tile threshold (PSX_AB_T128)
set -o pipefail
mkdir -p gpurun_out
for alt in "PSX_AB_WQT=512" "PSX_AB_RCW=512" "PSX_AB_T128=1024" "PSX_AB_T128=256"; do
  tag=${alt#PSX_AB_}
  bash scripts/prof/r6_ab.sh "PSX_X=0" "$alt" --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/g2_fp32_$tag.jsonl
  bash scripts/prof/r6_ab.sh "PSX_X=0" "$alt" --dtype bf16 --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/g2_bf16_$tag.jsonl
done
