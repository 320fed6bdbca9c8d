# kernel-trace profile of the ResNet-50 fp32 top-k sync step (BASELINE config 5 shape, N=1)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r50prof -o run -- python3 bench.py --model resnet50 --codec topk --steps 6 --warmup 3 --secondary none > gpurun_out/r50prof.log 2>&1 || { tail -5 gpurun_out/r50prof.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/r50prof/run_kernel_trace.csv --steps 5 > gpurun_out/r50prof.txt
python scripts/prof/kstats.py gpurun_out/r50prof/run_kernel_trace.csv --steps 5 --grid "conv2_kernel|wgrad" > gpurun_out/r50prof_grid.txt
head -40 gpurun_out/r50prof.txt
