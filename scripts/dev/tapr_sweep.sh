#!/bin/bash
# GPU-box helper: tap-reuse tile width sweep (fwd + dgrad), fp32 and bf16 layer benches.
set -o pipefail
OUT=gpurun_out/tsw
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_v2_gpu.py tests/test_fp32_gpu.py -k "fwd or dgrad or conv" > $OUT/tests.log 2>&1 || exit $?
for bn in 64 128 256; do
  PSX_CV_TAPR_BN=$bn ONLY=fwd MIOPEN=0 timeout -k 10 120 python bench/conv_layers_f32.py > $OUT/f32_fwd_$bn.jsonl 2>&1 || exit $?
  PSX_CV_TAPR_BN=$bn ONLY=dgrad MIOPEN=0 timeout -k 10 120 python bench/conv_layers_f32.py > $OUT/f32_dgrad_$bn.jsonl 2>&1 || exit $?
  PSX_CV_TAPR_BN=$bn timeout -k 10 200 python bench/conv_layers.py > $OUT/bf16_$bn.jsonl 2>&1 || exit $?
done
