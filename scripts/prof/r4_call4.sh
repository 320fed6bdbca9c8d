# fused wgrad: prefetch (default build) vs no-prefetch variant per layer, the fold bit-equality test,
# fused-wgrad tests, same-box bench A/B (WGF on/off), deterministic-mode A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wino_wgrad_gpu.py "tests/test_wino_gpu.py::test_engine_bn_fold_matches_unfolded" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c4_t.log 2>&1
rc=$?; tail -4 gpurun_out/c4_t.log
Q="16,32,64" timeout -k 10 300 python bench/wino_wgrad_ab.py | tee gpurun_out/wgf_ab_pf1.jsonl || exit 1
PSX_KERNELS_LIB=$PWD/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_wgfpf0.so Q="16,32,64" timeout -k 10 300 python bench/wino_wgrad_ab.py | tee gpurun_out/wgf_ab_pf0.jsonl || exit 1
AB_CFGS="PSX_WINO_WGF=0 PSX_WINO_WGF=1" bash scripts/prof/ab_env.sh || exit 1
bash scripts/prof/det_ab.sh || exit 1
exit $rc
