# kernel-trace profile of the fp32 headline step: per-kernel table and per-grid table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sprof -o run -- python3 bench.py --steps 10 --warmup 5 --secondary none > gpurun_out/sprof.log 2>&1 || { tail -5 gpurun_out/sprof.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/sprof/run_kernel_trace.csv --steps 8 > gpurun_out/sprof.txt
python scripts/prof/kstats.py gpurun_out/sprof/run_kernel_trace.csv --steps 8 --grid "wino|conv2_kernel|wgrad2f|bn_" > gpurun_out/sprof_grid.txt
head -45 gpurun_out/sprof.txt
python scripts/prof/timeline.py gpurun_out/sprof/run_kernel_trace.csv --list > gpurun_out/sprof_timeline.txt
