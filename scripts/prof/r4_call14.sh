# ResNet-50 fp32 A/B: side stream on/off, weight-gradient share
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in _ PSX_WGRAD_STREAM=0 PSX_WG_SHARE=0.5; do
  if [ "$cfg" = "_" ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 300 python bench.py --model resnet50 --codec topk --steps 8 --warmup 3 --secondary none > gpurun_out/r50ab.json 2>gpurun_out/r50ab.err || { tail -5 gpurun_out/r50ab.err; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r50ab.json)"
done
done
