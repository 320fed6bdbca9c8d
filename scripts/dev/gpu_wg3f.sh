#!/bin/bash
# GPU-box helper: fp32 tap-reuse weight-gradient sweep, per-layer fp32 conv bench vs MIOpen, PMC
# counters of the weight-gradient kernels and a kernel trace of the fp32 bench step.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/wg3f
mkdir -p $OUT
timeout -k 10 300 python bench/wgrad3f_sweep.py > $OUT/sweep.jsonl 2> $OUT/sweep.err || exit $?
timeout -k 10 300 python bench/conv_layers_f32.py > $OUT/layers.jsonl 2> $OUT/layers.err || exit $?
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
ONLY=wgrad MIOPEN=0 timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/pmc -o run -- \
  python bench/conv_layers_f32.py > $OUT/pmc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- \
  python bench.py --steps 15 --warmup 3 --secondary none > $OUT/prof.log 2>&1 || exit $?
