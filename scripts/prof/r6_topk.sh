# round 6: kernel trace of the R18 fp32 step with the top-k codec
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6tk -o run -- python3 bench.py --codec topk --steps 10 --warmup 5 --secondary none > gpurun_out/r6tk.log 2>&1 || { tail -5 gpurun_out/r6tk.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/r6tk/run_kernel_trace.csv --steps 8 > gpurun_out/r6tk.txt
python scripts/prof/kstats.py gpurun_out/r6tk/run_kernel_trace.csv --steps 8 --grid "tk_|topk" > gpurun_out/r6tk_grid.txt
rm -rf gpurun_out/r6tk
