# fp32 128x128 conv tiles + bgemm cfg4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/f32_tiles.py > gpurun_out/f32_tiles.jsonl 2>&1 || { tail -5 gpurun_out/f32_tiles.jsonl; exit 1; }
cat gpurun_out/f32_tiles.jsonl
timeout -k 10 200 python bench/bgemm_f32.py > gpurun_out/bgemm.jsonl 2>&1 || { tail -5 gpurun_out/bgemm.jsonl; exit 1; }
cat gpurun_out/bgemm.jsonl
