# convergence parity with the round-4 defaults (serial fp32 step, two graph queues)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/convergence_parity.py --out gpurun_out/convergence > gpurun_out/convergence.log 2>&1 || { tail -20 gpurun_out/convergence.log; exit 1; }
tail -25 gpurun_out/convergence.log
