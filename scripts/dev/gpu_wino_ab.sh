#!/bin/bash
# GPU-box helper: Winograd path tests + per-layer bench (default and PSX_WINO_WBR=128) + same-box
# bench.py A/B (default / PSX_WINO_WGRAD=0 / PSX_WINO=0). Usage: bash scripts/dev/gpu_wino_ab.sh
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py tests/test_fp32_gpu.py -v -s --timeout 200 --timeout-method thread > gpurun_out/wino_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/wino_tests.log | tail -30; exit 1; }
tail -3 gpurun_out/wino_tests.log
MIOPEN=0 timeout -k 10 300 python bench/conv_layers_f32.py > gpurun_out/wino_layers.jsonl 2> gpurun_out/wino_layers.err || exit 2
PSX_WINO_WBR=128 MIOPEN=0 timeout -k 10 300 python bench/conv_layers_f32.py > gpurun_out/wino_layers_wbr128.jsonl 2>> gpurun_out/wino_layers.err || exit 2
for v in def PSX_WINO_WGRAD=0 PSX_WINO=0 def PSX_WINO_WGRAD=0 PSX_WINO=0; do
  if [ $v = def ]; then e=PSX_DUMMY=1; else e=$v; fi
  env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --secondary none > gpurun_out/wino_bench.log 2>&1 || exit 3
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/wino_bench.log | sed "s/^/$v /"
done
