# counted-wait LDS fragment reads (PSX_CONV_ASMRD=1 variant library): GPU numerics, per-layer and headline A/B
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_asm1.so
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
PSX_KERNELS_LIB=$V timeout -k 10 600 $T tests -m gpu --ignore tests/test_multirank_gpu.py --ignore tests/test_elastic_gpu.py > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
timeout -k 10 300 python bench/f32_tiles.py > gpurun_out/f32_tiles_asm0.jsonl 2>&1 || { tail -5 gpurun_out/f32_tiles_asm0.jsonl; exit 1; }
PSX_KERNELS_LIB=$V timeout -k 10 300 python bench/f32_tiles.py > gpurun_out/f32_tiles_asm1.jsonl 2>&1 || { tail -5 gpurun_out/f32_tiles_asm1.jsonl; exit 1; }
timeout -k 10 300 python bench/r50_wgrad_f32.py > gpurun_out/r50_wgrad_asm0.jsonl 2>&1 || exit 1
PSX_KERNELS_LIB=$V timeout -k 10 300 python bench/r50_wgrad_f32.py > gpurun_out/r50_wgrad_asm1.jsonl 2>&1 || exit 1
AB_CFGS="_ PSX_KERNELS_LIB=$V" bash scripts/prof/ab_env.sh || exit 1
for rep in 1 2; do for cfg in _ PSX_KERNELS_LIB=$V; do
  if [ "$cfg" = "_" ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 200 python bench.py --dtype bf16 --steps 30 --warmup 10 --secondary none > gpurun_out/abh.json 2>gpurun_out/abh.err || { tail -5 gpurun_out/abh.err; exit 1; }
  echo "bf16 $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abh.json)"
done; done
for p in 0; do PSX_KERNELS_LIB=$V BN=128 timeout -k 10 60 python scripts/prof/sk_probe.py || exit 1; done
