#!/bin/bash
# GPU-box helper: PMC counters of the fp32 and bf16 conv / wgrad kernels on the per-layer benches
# (eager launches, no graphs). One rocprofv3 pass per counter group, each under its own limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
MIOPEN=0 timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/f32 -o run -- \
  python bench/conv_layers_f32.py > $OUT/f32.log 2>&1 || exit $?
MIOPEN=0 timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/bf16 -o run -- \
  python bench/conv_layers.py > $OUT/bf16.log 2>&1 || exit $?
