#!/bin/bash
# GPU-box helper: headline bench (fp32 and bf16) + a rocprofv3 kernel-trace of the fp32 step.
# Usage (from the repo root on the box): bash scripts/dev/gpu_bench_prof.sh [tag]
set -o pipefail
TAG=${1:-run}
ROOT=$(pwd)
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_fp32.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --dtype bf16 > gpurun_out/${TAG}_bench_bf16.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_$TAG -o run -- \
  python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_prof_fp32.log 2>&1 || exit $?
