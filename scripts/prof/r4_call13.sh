set -o pipefail
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 200 $T tests/test_sk_gemm_gpu.py > gpurun_out/t_sk.log 2>&1 || { tail -30 gpurun_out/t_sk.log; exit 1; }
tail -2 gpurun_out/t_sk.log
for p in 0 4 5; do PSX_SK_PROBE=$p BN=128 timeout -k 10 60 python scripts/prof/sk_probe.py || exit 1; done
