# forward shortcut fold (PSX_FWD_FOLD_SC) + unrolled head loops: numerics, engine tests, A/B, profile
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_fp32_gpu.py tests/test_kernels_gpu.py tests/test_conv_v2_gpu.py tests/test_deterministic_gpu.py tests/test_engine_gpu.py tests/test_resnet50_gpu.py > gpurun_out/t_ffold.log 2>&1 || { tail -30 gpurun_out/t_ffold.log; exit 1; }
tail -1 gpurun_out/t_ffold.log
AB_CFGS="_ PSX_FWD_FOLD_SC=0" bash scripts/prof/ab_env.sh || exit 1
for rep in 1 2 3; do
for cfg in _ PSX_FWD_FOLD_SC=0; do
  if [ "$cfg" = "_" ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 200 python bench.py --steps 30 --warmup 10 --dtype bf16 --secondary none > gpurun_out/abh.json 2>gpurun_out/abh.err || { tail -5 gpurun_out/abh.err; exit 1; }
  echo "bf16 $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abh.json)"
done
done
bash scripts/prof/step_prof.sh > /dev/null || exit 1
grep -E "head|conv2_kernel<float, 64, (64|128), 0, false, false" gpurun_out/sprof.txt
