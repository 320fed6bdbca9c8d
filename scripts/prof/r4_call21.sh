set -o pipefail
AB_CFGS="_ PSX_WGRAD_STREAM=0 PSX_WGRAD_STREAM=0,DEBUG_HIP_FORCE_GRAPH_QUEUES=2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2" bash scripts/prof/ab_env.sh || exit 1
for rep in 1 2; do for cfg in _ DEBUG_HIP_FORCE_GRAPH_QUEUES=2 PSX_WGRAD_STREAM=0 PSX_WGRAD_STREAM=0,DEBUG_HIP_FORCE_GRAPH_QUEUES=2 DEBUG_HIP_FORCE_GRAPH_QUEUES=3; do
  if [ "$cfg" = "_" ]; then envs=""; else envs="${cfg//,/ }"; fi
  env $envs timeout -k 10 200 python bench.py --dtype bf16 --steps 30 --warmup 10 --secondary none > gpurun_out/abh.json 2>gpurun_out/abh.err || { tail -5 gpurun_out/abh.err; exit 1; }
  echo "bf16 $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abh.json)"
done; done
for cfg in DEBUG_HIP_FORCE_GRAPH_QUEUES=2 _; do
  if [ "$cfg" = "_" ]; then envs=""; else envs="${cfg//,/ }"; fi
  env $envs timeout -k 10 300 python bench.py --model resnet50 --codec topk --steps 8 --warmup 3 --secondary none > gpurun_out/r50ab.json 2>gpurun_out/r50ab.err || { tail -5 gpurun_out/r50ab.err; exit 1; }
  echo "r50 $cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r50ab.json)"
done
