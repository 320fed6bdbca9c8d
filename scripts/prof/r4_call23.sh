set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_fp32_gpu.py tests/test_wino_gpu.py tests/test_wino_fused_gpu.py tests/test_deterministic_gpu.py tests/test_native_loop_gpu.py > gpurun_out/t_sub.log 2>&1 || { tail -30 gpurun_out/t_sub.log; exit 1; }
tail -2 gpurun_out/t_sub.log
AB_CFGS="_ PSX_WINO_WSTREAM=0" bash scripts/prof/ab_env.sh || exit 1
