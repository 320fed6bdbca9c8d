set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_wino_fused_gpu.py tests/test_wino_gpu.py tests/test_fp32_gpu.py tests/test_deterministic_gpu.py tests/test_engine_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ws_t.log 2>&1 || { tail -30 gpurun_out/ws_t.log; exit 1; }
tail -1 gpurun_out/ws_t.log
for rep in 1 2; do
for f in 0 1; do
  PSX_WINO_WSPLIT=$f timeout -k 10 200 python bench.py --steps 30 --warmup 10 --secondary none > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "WSPLIT=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
done
done
bash scripts/prof/step_prof.sh > /dev/null 2>&1 || { tail -5 gpurun_out/sprof.log; exit 1; }
head -12 gpurun_out/sprof.txt
grep wino_w_multi gpurun_out/sprof.txt
