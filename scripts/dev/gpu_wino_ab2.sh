#!/bin/bash
# GPU-box helper: Winograd tests, per-layer bench with weight-gradient split variants, and a
# same-box bench.py A/B of env variants given as arguments (default first and last).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/wino_tests.log 2>&1 || { tail -30 gpurun_out/wino_tests.log; exit 1; }
tail -1 gpurun_out/wino_tests.log
for wq in 0 2 8; do
  PSX_WINO_WQ=$wq MIOPEN=0 timeout -k 10 300 python bench/conv_layers_f32.py > gpurun_out/wino_layers_wq$wq.jsonl 2>> gpurun_out/wino_layers.err || exit 2
done
for v in def "$@" def; do
  if [ $v = def ]; then e=PSX_DUMMY=1; else e=$v; fi
  env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --secondary none > gpurun_out/wino_bench.log 2>&1 || exit 3
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/wino_bench.log | sed "s/^/$v /"
done
