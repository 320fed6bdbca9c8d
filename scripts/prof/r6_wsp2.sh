# round 6: bf16 weight-gradient split caps 256 -> 512 (wplan, wplanf) vs the base build
set -o pipefail
mkdir -p gpurun_out
BASE=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/libpsx_kernels_base.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_v2_gpu.py tests/test_engine_gpu.py -k "wgrad or step or engine" > gpurun_out/wsp2_tests.log 2>&1 || { tail -30 gpurun_out/wsp2_tests.log; exit 1; }
tail -1 gpurun_out/wsp2_tests.log
for cfg in "r50_fp32:--model resnet50 --codec topk --steps 10 --warmup 3" "r50_bf16:--model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3" "r18_fp32:" "r18_bf16:--dtype bf16"; do
  name=${cfg%%:*}; args=${cfg#*:}
  bash scripts/prof/r6_ab.sh "PSX_KERNELS_LIB=$BASE" "PSX_X=1" $args || exit 1
  cp gpurun_out/ab.jsonl gpurun_out/wsp2_ab_$name.jsonl
done
