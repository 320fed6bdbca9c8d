# top-k probe: pass A without the global-histogram atomics, pass B without the coarse LDS histogram (wrong results)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for pr in 0 4 2; do
  n=11220132
  PSX_AB_TKPROBE=$pr timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tk4 -o run -- python3 bench/topk_bench.py --n $n --dtype fp32 > gpurun_out/tk7_${pr}.log 2>&1 || { tail -5 gpurun_out/tk7_${pr}.log; exit 1; }
  python scripts/prof/kstats.py gpurun_out/tk4/run_kernel_trace.csv --steps 20 --marker tk_pass_a > gpurun_out/tk7_${pr}.txt
  rm -rf gpurun_out/tk4
done
