set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_deterministic_gpu.py tests/test_engine_gpu.py tests/test_fp32_gpu.py tests/test_wino_gpu.py tests/test_wino_fused_gpu.py tests/test_ps_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tl_t.log 2>&1 || { tail -30 gpurun_out/tl_t.log; exit 1; }
tail -1 gpurun_out/tl_t.log
AB_CFGS="PSX_TAIL_SPLIT=0 PSX_TAIL_SPLIT=1" bash scripts/prof/ab_env.sh
