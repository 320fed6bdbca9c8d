# fused Winograd kernel: per-layer timing of A/B / diagnostic builds (_native/variants)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/wf_probe.jsonl
for v in base ${WF_VARIANTS:-apf p1 p2 p4 p8 p15}; do
  lib=""
  [ "$v" != base ] && lib="$PWD/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_$v.so"
  PSX_KERNELS_LIB=$lib timeout -k 10 120 python -u bench/wino_fused_ab.py > gpurun_out/wf_probe_$v.jsonl 2>&1 || { tail -5 gpurun_out/wf_probe_$v.jsonl; exit 1; }
  sed "s/^{/{\"variant\": \"$v\", /" gpurun_out/wf_probe_$v.jsonl | grep variant >> gpurun_out/wf_probe.jsonl
done
cat gpurun_out/wf_probe.jsonl
