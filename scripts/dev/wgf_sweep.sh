#!/bin/bash
# GPU-box helper: fp32 weight-gradient plan A/B (default plan vs forced splits), interleaved
# twice to expose order effects (first process on a fresh box).
set -o pipefail
OUT=gpurun_out/wgf
mkdir -p $OUT
for rep in 1 2; do
  ONLY=wgrad MIOPEN=0 timeout -k 10 120 python bench/conv_layers_f32.py > $OUT/default_$rep.jsonl 2>&1 || exit $?
  for sp in 28 84; do
    PSX_WGF_BR=64 PSX_WGF_BC=64 PSX_WGF_SPLITS=$sp ONLY=wgrad MIOPEN=0 \
      timeout -k 10 120 python bench/conv_layers_f32.py > $OUT/s64_${sp}_$rep.jsonl 2>&1 || exit $?
  done
done
