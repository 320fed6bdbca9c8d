# round 6: bf16 / fp32 ResNet-18 step timelines (queue overlap, last step's kernel order)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --dtype bf16 --steps 10 --warmup 5 --secondary none > gpurun_out/tl.log 2>&1 || { tail -5 gpurun_out/tl.log; exit 1; }
python scripts/prof/timeline.py gpurun_out/tl/run_kernel_trace.csv --steps 8 --list > gpurun_out/r6_bf16_timeline.txt
rm -rf gpurun_out/tl
