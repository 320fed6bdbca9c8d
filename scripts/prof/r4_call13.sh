set -o pipefail
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 200 $T tests/test_sk_gemm_gpu.py > gpurun_out/t_sk.log 2>&1 || { tail -30 gpurun_out/t_sk.log; exit 1; }
tail -2 gpurun_out/t_sk.log
for p in 0 4; do for bn in 128 64; do PSX_SK_PROBE=$p BN=$bn timeout -k 10 60 python scripts/prof/sk_probe.py || exit 1; done; done
for bn in 128 64; do SHAPE=128,512,512,36 BN=$bn timeout -k 10 60 python scripts/prof/sk_probe.py | sed "s/^/L4 /"|| exit 1; done
