# direct stem conv v2 (scalar-register weights): probe, numerics, A/B fp32 + bf16
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench/stem_probe.py > gpurun_out/stem_probe.jsonl 2>&1 || { tail -5 gpurun_out/stem_probe.jsonl; exit 1; }
grep -E "direct|plan" gpurun_out/stem_probe.jsonl
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_fp32_gpu.py tests/test_conv_v2_gpu.py -k "stem" > gpurun_out/t_stem.log 2>&1 || { tail -30 gpurun_out/t_stem.log; exit 1; }
tail -1 gpurun_out/t_stem.log
AB_CFGS="_ PSX_STEM_DIRECT=0" bash scripts/prof/ab_env.sh || exit 1
for rep in 1 2 3; do
for cfg in _ PSX_STEM_DIRECT=0; do
  if [ "$cfg" = "_" ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 200 python bench.py --steps 30 --warmup 10 --dtype bf16 --secondary none > gpurun_out/abh.json 2>gpurun_out/abh.err || { tail -5 gpurun_out/abh.err; exit 1; }
  echo "bf16 $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abh.json)"
done
done
