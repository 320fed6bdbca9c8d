# fused Winograd: kernel tests, engine tests with the fused path on, then a same-box bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wino_fused_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wf_t.log 2>&1 || { tail -30 gpurun_out/wf_t.log; exit 1; }
tail -2 gpurun_out/wf_t.log
PSX_WINO_FUSE=1 timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py tests/test_fp32_gpu.py tests/test_deterministic_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wf_e.log 2>&1 || { tail -30 gpurun_out/wf_e.log; exit 1; }
tail -2 gpurun_out/wf_e.log
timeout -k 10 200 python -u bench/wino_fused_ab.py > gpurun_out/wf_ab.jsonl 2>&1 || { tail -20 gpurun_out/wf_ab.jsonl; exit 1; }
cat gpurun_out/wf_ab.jsonl
for rep in 1 2; do
for f in 0 1; do
  PSX_WINO_FUSE=$f timeout -k 10 200 python bench.py --steps 30 --warmup 10 --secondary none > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "FUSE=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
done
done
