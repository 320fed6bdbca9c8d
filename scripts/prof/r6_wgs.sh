# round 6: side-stream weight gradients re-checked on the final kernels (PSX_TUNE wgrad_stream)
set -o pipefail
mkdir -p gpurun_out
bash scripts/prof/r6_ab.sh "PSX_X=0" "PSX_TUNE=wgrad_stream=1" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wgs_fp32.jsonl
bash scripts/prof/r6_ab.sh "PSX_X=0" "PSX_TUNE=wgrad_stream=0" --dtype bf16 --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wgs_bf16.jsonl
