#!/bin/bash
# GPU-box helper: engine-step A/B vs MIOpen (bf16 / fp32) and the ResNet-50 top-k benches + profile.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r50
mkdir -p $OUT
timeout -k 10 200 python bench/engine_step.py --dtype bf16 > $OUT/engine_bf16.json 2>&1 || exit $?
timeout -k 10 200 python bench/engine_step.py --dtype fp32 > $OUT/engine_fp32.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3 --secondary none > $OUT/r50_topk_bf16.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python bench.py --model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3 --secondary none > $OUT/r50_prof.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model resnet50 --codec topk --steps 10 --warmup 3 --secondary none > $OUT/r50_topk_fp32.log 2>&1 || exit $?
