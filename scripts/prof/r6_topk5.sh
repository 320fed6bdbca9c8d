# top-k encode geometry A/B: 256 chunks x 1024 threads (geo 1) vs 1024 x 256 (geo 0); tests under both
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for geo in 1; do
  PSX_AB_TKGEO=$geo timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_topk_gpu.py tests/test_elastic_gpu.py tests/test_rccl_native_gpu.py > gpurun_out/tk8_tests$geo.log 2>&1 || { tail -30 gpurun_out/tk8_tests$geo.log; exit 1; }
  tail -1 gpurun_out/tk8_tests$geo.log
  for n in 11220132 25557032; do
    PSX_AB_TKGEO=$geo timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tk4 -o run -- python3 bench/topk_bench.py --n $n --dtype fp32 > gpurun_out/tk8_${geo}_$n.log 2>&1 || { tail -5 gpurun_out/tk8_${geo}_$n.log; exit 1; }
    python scripts/prof/kstats.py gpurun_out/tk4/run_kernel_trace.csv --steps 20 --marker tk_pass_a > gpurun_out/tk8_${geo}_$n.txt
    rm -rf gpurun_out/tk4
  done
  PSX_AB_TKGEO=$geo timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tk2 -o run -- python3 bench.py --codec topk --steps 10 --warmup 5 --secondary none > gpurun_out/tk2.log 2>&1 || { tail -5 gpurun_out/tk2.log; exit 1; }
  python scripts/prof/kstats.py gpurun_out/tk2/run_kernel_trace.csv --steps 8 > gpurun_out/tk8_${geo}_step.txt
  rm -rf gpurun_out/tk2
done
