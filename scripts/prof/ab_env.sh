# same-box A/B of the fp32 headline over env settings: AB_CFGS="NAME=a NAME=b" (use _ for none)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for cfg in ${AB_CFGS}; do
  if [ "$cfg" = "_" ]; then envs=""; else envs="${cfg//,/ }"; fi
  env $envs timeout -k 10 200 python bench.py --steps 30 --warmup 10 --secondary none > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
done
done
