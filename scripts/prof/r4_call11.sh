# stream-K Winograd GEMM: numerics, GEMM bench, headline A/B
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 200 $T tests/test_sk_gemm_gpu.py > gpurun_out/t_sk.log 2>&1 || { tail -30 gpurun_out/t_sk.log; exit 1; }
tail -2 gpurun_out/t_sk.log
timeout -k 10 300 $T tests/test_wino_gpu.py tests/test_fp32_gpu.py > gpurun_out/t_wino.log 2>&1 || { tail -30 gpurun_out/t_wino.log; exit 1; }
tail -2 gpurun_out/t_wino.log
timeout -k 10 200 python bench/bgemm_f32.py > gpurun_out/bgemm.jsonl 2>&1 || { tail -5 gpurun_out/bgemm.jsonl; exit 1; }
cat gpurun_out/bgemm.jsonl
AB_CFGS="_ PSX_WINO_SK=0" bash scripts/prof/ab_env.sh || exit 1
