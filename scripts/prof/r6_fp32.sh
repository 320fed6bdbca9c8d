# round 6: kernel trace of the fp32 (headline) and bf16 ResNet-18 steps and the ResNet-50 top-k steps
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name, bench args
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$1 -o run -- python3 bench.py --secondary none "${@:2}" > gpurun_out/$1.log 2>&1 || { tail -5 gpurun_out/$1.log; exit 1; }
  python scripts/prof/kstats.py gpurun_out/$1/run_kernel_trace.csv --steps ${STEPS:-8} > gpurun_out/$1_kernels.txt
  python scripts/prof/kstats.py gpurun_out/$1/run_kernel_trace.csv --steps ${STEPS:-8} --grid "conv2|wgrad|wino|bn_|head|tk_" > gpurun_out/$1_kernels_by_grid.txt
  rm -rf gpurun_out/$1
}
run r6_r18_fp32 --steps 10 --warmup 5 || exit 1
run r6_r18_bf16 --dtype bf16 --steps 10 --warmup 5 || exit 1
STEPS=4 run r6_r50_fp32 --model resnet50 --codec topk --steps 5 --warmup 3 || exit 1
STEPS=4 run r6_r50_bf16 --model resnet50 --codec topk --dtype bf16 --steps 5 --warmup 3 || exit 1
