# round 6: BN apply passes' workgroup cap (each workgroup recomputes the finalize; PSX_AB_FINCAP) step A/B
set -o pipefail
mkdir -p gpurun_out
for c in 512 256; do
  bash scripts/prof/r6_ab.sh "PSX_AB_FINCAP=1024" "PSX_AB_FINCAP=$c" --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/fincap_fp32_$c.jsonl
  bash scripts/prof/r6_ab.sh "PSX_AB_FINCAP=1024" "PSX_AB_FINCAP=$c" --dtype bf16 --steps 30 --warmup 10 || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/fincap_bf16_$c.jsonl
done
