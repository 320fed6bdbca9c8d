# round 6: the late-round kernel tuning (weight-gradient split caps / stages, split-K epilogue,
# Winograd transform grid, BN apply cap) against the kernel library of commit 3a74c8c, same box
set -o pipefail
mkdir -p gpurun_out
BASE=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/libpsx_kernels_base.so
for cfg in "r18_fp32:" "r18_bf16:--dtype bf16" "r50_fp32:--model resnet50 --codec topk --steps 10 --warmup 3" "r50_bf16:--model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3"; do
  name=${cfg%%:*}; args=${cfg#*:}
  bash scripts/prof/r6_ab.sh "PSX_KERNELS_LIB=$BASE" "PSX_X=1" $args || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/sess_ab_$name.jsonl
done
