#!/usr/bin/env bash
# Experiment matrix on one MI355X node: sync and async PS at 1/2/4/8 GPUs (rank 0 = server),
# METRICS_JSON logs -> experiment_results/*.json -> plots/ (replaces the reference's
# terraform apply + CloudWatch parse + visualise loop, EXPERIMENT_GUIDE.md).
#
#   deploy/run_experiments.sh [epochs] [gpu counts...]      e.g.  deploy/run_experiments.sh 3 1 2 4 8
set -euo pipefail
cd "$(dirname "$0")/.."
EPOCHS=${1:-3}; shift || true
GPUS=${*:-"1 2 4 8"}
export HSA_ENABLE_IPC_MODE_LEGACY=0
python csrc/build.py
mkdir -p runs experiment_results plots
for mode in sync async; do
  for n in $GPUS; do
    name="${mode}_${n}workers"
    timeout -k 10 3600 python scripts/launch.py --nproc "$n" --log "runs/${name}.log" -- \
      --mode "$mode" --epochs "$EPOCHS" --workers "$n" --log-dir "runs/${name}"
    python scripts/parse_logs.py "runs/${name}.log" --experiment-name "$name" \
      --output "experiment_results/${name}.json"
  done
done
: > runs/bench_scaling.jsonl
for n in $GPUS; do
  timeout -k 10 1200 python scripts/launch.py --bench --nproc "$n" -- --steps 50 --warmup 10 \
    | grep '^{' | tail -n 1 >> runs/bench_scaling.jsonl
done
python scripts/visualize_results.py --results-dir experiment_results --bench runs/bench_scaling.jsonl \
  --output-dir plots
