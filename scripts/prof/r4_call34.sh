# max-pool backward as a 2x2-block gather: numerics, probe, ResNet-50 fp32 step
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_fp32_gpu.py tests/test_resnet50_gpu.py -k "maxpool" > gpurun_out/t_pool.log 2>&1 || { tail -30 gpurun_out/t_pool.log; exit 1; }
tail -1 gpurun_out/t_pool.log
timeout -k 10 120 python bench/pool_probe.py > gpurun_out/pool_probe.jsonl 2>&1 || { tail -5 gpurun_out/pool_probe.jsonl; exit 1; }
grep dtype gpurun_out/pool_probe.jsonl
timeout -k 10 400 python bench.py --model resnet50 --steps 10 --warmup 3 --secondary none > gpurun_out/r50.json 2> gpurun_out/r50.err || { tail -5 gpurun_out/r50.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r50.json
