# round 6: end-to-end result artifacts on the current engine (fp32 HIP engine, synthetic CIFAR-100
# shape, one MI355X): sync W=1 3 epochs (reference BN semantics and --bn-sync), async W=7 worker
# threads; each run's METRICS_JSON aggregated into the reference's experiment_results schema.
set -o pipefail
mkdir -p gpurun_out/r6_art
A=gpurun_out/r6_art
timeout -k 10 300 python scripts/psx_train.py --mode sync --workers 1 --epochs 3 --synthetic --eval-every 1 --log-dir $A/sync_w1 > $A/sync_w1.log 2>&1
timeout -k 10 300 python scripts/psx_train.py --mode sync --workers 1 --epochs 3 --synthetic --eval-every 1 --bn-sync --log-dir $A/sync_w1_bnsync > $A/sync_w1_bnsync.log 2>&1
timeout -k 10 300 python bench/async_staleness.py --workers 7 --steps 60 --out-dir $A/async > $A/async.log 2>&1
python scripts/parse_logs.py --experiment-name sync_1worker_r6 --output $A/sync_1worker_r6.json $A/sync_w1 > /dev/null
python scripts/parse_logs.py --experiment-name sync_1worker_bnsync_r6 --output $A/sync_1worker_bnsync_r6.json $A/sync_w1_bnsync > /dev/null
