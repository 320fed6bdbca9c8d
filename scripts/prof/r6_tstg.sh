# round 6: tap-reuse LDS ring depth A/B (2 vs 3 stages) — correctness, per-layer, in-step
set -o pipefail
mkdir -p gpurun_out
for n in 3 2; do
  PSX_AB_TSTG=$n timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_v2_gpu.py -k "tap_reuse or conv2" > gpurun_out/tstg_test$n.log 2>&1 || { tail -20 gpurun_out/tstg_test$n.log; exit 1; }
  tail -1 gpurun_out/tstg_test$n.log
done
for n in 2 3; do
  PSX_AB_TSTG=$n timeout -k 10 200 python bench/conv_layers.py > gpurun_out/tstg_layers$n.jsonl 2>/dev/null || exit 1
done
bash scripts/prof/r6_ab.sh "PSX_AB_TSTG=2" "PSX_AB_TSTG=3" --dtype bf16 --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/tstg_ab_bf16.jsonl
bash scripts/prof/r6_ab.sh "PSX_AB_TSTG=2" "PSX_AB_TSTG=3" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/tstg_ab_fp32.jsonl
