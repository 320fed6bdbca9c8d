#!/bin/bash
# GPU-box helper: same-box A/B of kernel-library variants (csrc/build.py --variant NAME ...):
# fp32 per-layer conv bench and the fp32 bench step for the default build and each variant.
# Usage: bash scripts/dev/gpu_variant_ab.sh TAG VARIANT...   (VARIANT = a build name, or
# env:NAME=VALUE to run the default build with that environment variable set); DTYPE=bf16 runs
# the bf16 layer bench and bench.py --dtype bf16 instead
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
OUT=gpurun_out/$T
mkdir -p $OUT
V=distributed-parameter-server-for-ml-training_amd/_native/variants
for v in default "$@" default; do
  unset PSX_KERNELS_LIB
  case "$v" in
    default) ;;
    env:*) export "${v#env:}" ;;
    *) export PSX_KERNELS_LIB=$PWD/$V/libpsx_kernels_$v.so ;;
  esac
  if [ "${DTYPE:-fp32}" = bf16 ]; then
    timeout -k 10 300 python bench/conv_layers.py > $OUT/layers_$v.jsonl 2> $OUT/layers_$v.err || exit $?
  else
    MIOPEN=0 timeout -k 10 300 python bench/conv_layers_f32.py > $OUT/layers_$v.jsonl 2> $OUT/layers_$v.err || exit $?
  fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --secondary none --dtype ${DTYPE:-fp32} >> $OUT/bench_$v.log 2>&1 || exit $?
  case "$v" in env:*) unset "$(echo ${v#env:} | cut -d= -f1)" ;; esac
done
