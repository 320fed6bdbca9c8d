# round 6: split-K epilogue workgroup count (PSX_AB_EPPB = target workgroups) with batched slab loads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_v2_gpu.py tests/test_fp32_gpu.py tests/test_kernels_gpu.py > gpurun_out/epi_tests.log 2>&1 || { tail -30 gpurun_out/epi_tests.log; exit 1; }
tail -1 gpurun_out/epi_tests.log
for e in 512 128 64 32; do
  PSX_AB_EPPB=$e timeout -k 10 200 python bench/conv_layers.py > gpurun_out/epi_layers_$e.jsonl 2>/dev/null || exit 1
done
bash scripts/prof/r6_ab.sh "PSX_AB_EPPB=512" "PSX_AB_EPPB=64" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/epi_ab_fp32.jsonl
bash scripts/prof/r6_ab.sh "PSX_AB_EPPB=512" "PSX_AB_EPPB=64" --dtype bf16 --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/epi_ab_bf16.jsonl
