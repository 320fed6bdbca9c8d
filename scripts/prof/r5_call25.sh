# round 5 call 25: kernel tables of the round-5 tree (R18 fp32 / bf16, R50 bf16 / fp32)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {  # name, steps, bench args...
  n=$1; st=$2; shift 2
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k_$n -o run -- python3 bench.py "$@" --steps $st --warmup 3 --secondary none > gpurun_out/k_$n.log 2>&1 || { tail -5 gpurun_out/k_$n.log; return 1; }
  python scripts/prof/kstats.py gpurun_out/k_$n/run_kernel_trace.csv --steps $st > gpurun_out/r5c25_$n.txt
  python scripts/prof/kstats.py gpurun_out/k_$n/run_kernel_trace.csv --steps $st --grid "conv2_kernel|wgrad|bn_|stem|wino" > gpurun_out/r5c25_${n}_by_grid.txt
  rm -rf gpurun_out/k_$n
  head -14 gpurun_out/r5c25_$n.txt
}
prof r18_fp32 10 --dtype fp32 && prof r18_bf16 10 --dtype bf16 && prof r50_bf16 5 --model resnet50 --codec topk --dtype bf16 && prof r50_fp32 5 --model resnet50 --codec topk --dtype fp32
