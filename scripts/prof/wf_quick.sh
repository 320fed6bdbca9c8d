# fused Winograd kernel: GPU tests + per-layer A/B (bench/wino_fused_ab.py); WF_VARIANTS="a b" also tests and times
# _native/variants/libpsx_kernels_<v>.so builds (csrc/build.py build_variant)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wino_fused_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wf_t.log 2>&1 || { tail -30 gpurun_out/wf_t.log; exit 1; }
tail -1 gpurun_out/wf_t.log
timeout -k 10 200 python -u bench/wino_fused_ab.py > gpurun_out/wf_ab.jsonl 2>&1 || { tail -20 gpurun_out/wf_ab.jsonl; exit 1; }
cat gpurun_out/wf_ab.jsonl
for v in ${WF_VARIANTS:-}; do
  PSX_KERNELS_LIB=$PWD/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_$v.so timeout -k 10 300 python -u -m pytest tests/test_wino_fused_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wf_t_$v.log 2>&1 || { echo "== $v tests FAILED"; tail -20 gpurun_out/wf_t_$v.log; exit 1; }
  PSX_KERNELS_LIB=$PWD/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_$v.so timeout -k 10 120 python -u bench/wino_fused_ab.py > gpurun_out/wf_ab_$v.jsonl 2>&1 || { tail -5 gpurun_out/wf_ab_$v.jsonl; exit 1; }
  echo "== $v"; cat gpurun_out/wf_ab_$v.jsonl
done
