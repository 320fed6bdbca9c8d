# round 6: refinement of the two grid choices (BN apply cap 512 vs 384 / 768, Winograd transform grid 1024 vs 768)
set -o pipefail
mkdir -p gpurun_out
for alt in "PSX_AB_FINCAP=384" "PSX_AB_FINCAP=768" "PSX_AB_XFG=768"; do
  tag=${alt#PSX_AB_}
  bash scripts/prof/r6_ab.sh "PSX_X=0" "$alt" --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/ref_fp32_$tag.jsonl
  bash scripts/prof/r6_ab.sh "PSX_X=0" "$alt" --dtype bf16 --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/ref_bf16_$tag.jsonl
done
