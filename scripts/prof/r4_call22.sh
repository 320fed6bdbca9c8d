# new defaults: two graph queues (psx import), no weight-gradient side stream for fp32 CIFAR ResNet-18
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $T tests -m gpu --ignore tests/test_multirank_gpu.py --ignore tests/test_elastic_gpu.py > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
AB_CFGS="_ PSX_GRAPH_QUEUES=0,PSX_WGRAD_STREAM=1" bash scripts/prof/ab_env.sh || exit 1
for rep in 1 2; do for cfg in _ PSX_GRAPH_QUEUES=0; do
  if [ "$cfg" = "_" ]; then envs=""; else envs="${cfg//,/ }"; fi
  env $envs timeout -k 10 200 python bench.py --dtype bf16 --steps 30 --warmup 10 --secondary none > gpurun_out/abh.json 2>gpurun_out/abh.err || { tail -5 gpurun_out/abh.err; exit 1; }
  echo "bf16 $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abh.json)"
done; done
timeout -k 10 300 python bench.py --model resnet50 --codec topk --steps 8 --warmup 3 --secondary none > gpurun_out/r50ab.json 2>gpurun_out/r50ab.err || { tail -5 gpurun_out/r50ab.err; exit 1; }
echo "r50 default $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r50ab.json)"
