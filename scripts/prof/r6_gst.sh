# round 6: Winograd batched-GEMM reduction split threshold (PSX_AB_GST) step A/B, fp32
set -o pipefail
mkdir -p gpurun_out
for alt in "PSX_AB_GST=2048" "PSX_AB_GST=1"; do
  tag=${alt#PSX_AB_}
  bash scripts/prof/r6_ab.sh "PSX_X=0" "$alt" --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/gst_fp32_$tag.jsonl
done
