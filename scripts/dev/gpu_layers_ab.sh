#!/bin/bash
# GPU-box helper: conv kernel tests + fp32 / bf16 per-layer benches + the fp32 bench step.
set -o pipefail
export TMPDIR=/tmp
T=${1:-ab}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py tests/test_conv_v2_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
MIOPEN=0 timeout -k 10 300 python bench/conv_layers_f32.py > $OUT/layers_f32.jsonl 2> $OUT/layers_f32.err || exit $?
MIOPEN=0 timeout -k 10 300 python bench/conv_layers.py > $OUT/layers_bf16.jsonl 2> $OUT/layers_bf16.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
