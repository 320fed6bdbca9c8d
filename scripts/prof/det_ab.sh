# same-box A/B of deterministic mode (fixed-order BN reductions) vs the default, fp32 and bf16,
# interleaved; prints ms/step per run
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for dt in fp32 bf16; do
for det in 0 1; do
  PSX_DETERMINISTIC=$det timeout -k 10 200 python bench.py --steps 40 --warmup 10 --secondary none --dtype $dt > gpurun_out/det.json 2>gpurun_out/det.err || { tail -5 gpurun_out/det.err; exit 1; }
  echo "{\"dtype\": \"$dt\", \"deterministic\": $det, \"rep\": $rep, $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/det.json)}" | tee -a gpurun_out/det_ab.jsonl
done
done
done
