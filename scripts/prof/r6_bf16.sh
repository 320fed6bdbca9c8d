# round 6: bf16 step kernel trace, overlapped (default) and serial (PSX_TUNE wgrad_stream=0)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6b16 -o run -- python3 bench.py --dtype bf16 --steps 10 --warmup 5 --secondary none > gpurun_out/r6b16.log 2>&1 || { tail -5 gpurun_out/r6b16.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/r6b16/run_kernel_trace.csv --steps 8 > gpurun_out/r6b16.txt
python scripts/prof/kstats.py gpurun_out/r6b16/run_kernel_trace.csv --steps 8 --grid "conv2|wgrad|bn_|head|pool" > gpurun_out/r6b16_grid.txt
export PSX_TUNE=wgrad_stream=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6b16s -o run -- python3 bench.py --dtype bf16 --steps 10 --warmup 5 --secondary none > gpurun_out/r6b16s.log 2>&1 || { tail -5 gpurun_out/r6b16s.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/r6b16s/run_kernel_trace.csv --steps 8 --grid "conv2|wgrad|bn_|head|pool" > gpurun_out/r6b16s_grid.txt
rm -rf gpurun_out/r6b16 gpurun_out/r6b16s
