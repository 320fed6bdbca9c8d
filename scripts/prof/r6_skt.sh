# round 6: conv split-K plan (target workgroups PSX_AB_SKT, min k-steps per split PSX_AB_SKM) step A/B
set -o pipefail
mkdir -p gpurun_out
for alt in "PSX_AB_SKT=256" "PSX_AB_SKT=1024" "PSX_AB_SKM=4"; do
  tag=${alt#PSX_AB_}
  bash scripts/prof/r6_ab.sh "PSX_AB_SKT=512" "$alt" --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/skt_fp32_$tag.jsonl
  bash scripts/prof/r6_ab.sh "PSX_AB_SKT=512" "$alt" --dtype bf16 --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/skt_bf16_$tag.jsonl
done
