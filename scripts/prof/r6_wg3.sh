# round 6: wgrad3 with compile-time LDS stages (unrolled by NS) vs the base build (PSX_KERNELS_LIB)
set -o pipefail
mkdir -p gpurun_out
BASE=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/libpsx_kernels_base.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_v2_gpu.py -k "wgrad" > gpurun_out/wg3_tests.log 2>&1 || { tail -30 gpurun_out/wg3_tests.log; exit 1; }
tail -1 gpurun_out/wg3_tests.log
for rep in 1 2; do
  PSX_KERNELS_LIB=$BASE timeout -k 10 120 python bench/wgrad_probe.py --layers 1,4,7,10 > gpurun_out/wg3_base_$rep.txt 2>&1 || exit 1
  timeout -k 10 120 python bench/wgrad_probe.py --layers 1,4,7,10 > gpurun_out/wg3_new_$rep.txt 2>&1 || exit 1
done
bash scripts/prof/r6_ab.sh "PSX_KERNELS_LIB=$BASE" "PSX_X=1" --dtype bf16 --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wg3_ab_bf16.jsonl
