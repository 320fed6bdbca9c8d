#!/bin/bash
# GPU-box helper: per-layer fp32 conv timing vs MIOpen + counter list. Usage: bash scripts/dev/gpu_layers.sh TAG
set -o pipefail
TAG=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench/conv_layers_f32.py > gpurun_out/${TAG}_layers_f32.log 2>&1 || exit $?
timeout -k 10 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
