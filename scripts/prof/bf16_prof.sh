# kernel-trace profile of the bf16 step
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b16 -o run -- python3 bench.py --dtype bf16 --steps 10 --warmup 5 --secondary none > gpurun_out/b16.log 2>&1 || { tail -5 gpurun_out/b16.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/b16/run_kernel_trace.csv --steps 8 > gpurun_out/b16.txt
python scripts/prof/kstats.py gpurun_out/b16/run_kernel_trace.csv --steps 8 --grid "conv2|wgrad|bn_|head|pool" > gpurun_out/b16_grid.txt
head -30 gpurun_out/b16.txt
python scripts/prof/timeline.py gpurun_out/b16/run_kernel_trace.csv --list > gpurun_out/b16_timeline.txt
