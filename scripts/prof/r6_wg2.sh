# round 6: wgrad2 / wgrad2f with compile-time LDS stages + a 1x1/s1 identity fast path vs the base build
set -o pipefail
mkdir -p gpurun_out
BASE=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/libpsx_kernels_base.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_v2_gpu.py tests/test_wino_gpu.py tests/test_fp32_gpu.py tests/test_topk_gpu.py -k "wgrad or wino or topk or step" > gpurun_out/wg2_tests.log 2>&1 || { tail -30 gpurun_out/wg2_tests.log; exit 1; }
tail -1 gpurun_out/wg2_tests.log
bash scripts/prof/r6_ab.sh "PSX_KERNELS_LIB=$BASE" "PSX_X=1" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wg2_ab_r18_fp32.jsonl
bash scripts/prof/r6_ab.sh "PSX_KERNELS_LIB=$BASE" "PSX_X=1" --model resnet50 --codec topk --steps 10 --warmup 3 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wg2_ab_r50_fp32.jsonl
bash scripts/prof/r6_ab.sh "PSX_KERNELS_LIB=$BASE" "PSX_X=1" --model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wg2_ab_r50_bf16.jsonl
