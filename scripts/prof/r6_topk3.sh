# top-k encode: tests + per-kernel time at ResNet-18 / ResNet-50 gradient sizes + the R18 step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_topk_gpu.py > gpurun_out/tk6_tests.log 2>&1 || { tail -30 gpurun_out/tk6_tests.log; exit 1; }
tail -1 gpurun_out/tk6_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for n in 11220132 25557032; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tk4 -o run -- python3 bench/topk_bench.py --n $n --dtype fp32 > gpurun_out/tk6_$n.log 2>&1 || { tail -5 gpurun_out/tk6_$n.log; exit 1; }
  python scripts/prof/kstats.py gpurun_out/tk4/run_kernel_trace.csv --steps 20 --marker tk_pass_a > gpurun_out/tk6_$n.txt
  rm -rf gpurun_out/tk4
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tk2 -o run -- python3 bench.py --codec topk --steps 10 --warmup 5 --secondary none > gpurun_out/tk2.log 2>&1 || { tail -5 gpurun_out/tk2.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/tk2/run_kernel_trace.csv --steps 8 > gpurun_out/r6_topk_r18_kernels.txt
rm -rf gpurun_out/tk2
