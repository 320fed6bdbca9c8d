#!/bin/bash
# GPU-box helper: fp32 conv tile sweep (tap-reuse width, generic tiles) on the layer bench.
set -o pipefail
OUT=gpurun_out/f32sw
mkdir -p $OUT
for bn in 64 128 256; do
  PSX_CV_TAPR_BN=$bn ONLY=fwd MIOPEN=0 timeout -k 10 120 python bench/conv_layers_f32.py > $OUT/fwd_tapr$bn.jsonl 2>&1 || exit $?
  PSX_CV_TAPR_BN=$bn ONLY=dgrad MIOPEN=0 timeout -k 10 120 python bench/conv_layers_f32.py > $OUT/dgrad_tapr$bn.jsonl 2>&1 || exit $?
done
for cfg in "64 128 1" "64 256 1" "64 64 2" "64 128 2"; do
  set -- $cfg
  PSX_CV_TAPR=0 PSX_CV_BM=$1 PSX_CV_BN=$2 PSX_CV_WGM=$3 ONLY=fwd MIOPEN=0 timeout -k 10 120 python bench/conv_layers_f32.py > $OUT/fwd_g_$1_$2_$3.jsonl 2>&1 || exit $?
  PSX_CV_TAPR=0 PSX_CV_BM=$1 PSX_CV_BN=$2 PSX_CV_WGM=$3 ONLY=dgrad MIOPEN=0 timeout -k 10 120 python bench/conv_layers_f32.py > $OUT/dgrad_g_$1_$2_$3.jsonl 2>&1 || exit $?
done
