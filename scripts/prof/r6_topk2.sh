# round 6: top-k encode rework (256 x 1024-thread chunks, ballot ranks) — tests + kernel tables
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_topk_gpu.py tests/test_elastic_gpu.py -k "topk or encode or ties" > gpurun_out/tk2_tests.log 2>&1 || { tail -30 gpurun_out/tk2_tests.log; exit 1; }
tail -2 gpurun_out/tk2_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tk2 -o run -- python3 bench.py --codec topk --steps 10 --warmup 5 --secondary none > gpurun_out/tk2.log 2>&1 || { tail -5 gpurun_out/tk2.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/tk2/run_kernel_trace.csv --steps 8 > gpurun_out/r6_topk_r18_kernels.txt
rm -rf gpurun_out/tk2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tk3 -o run -- python3 bench/topk_bench.py --n 25557032 --dtype fp32 > gpurun_out/tk3.log 2>&1 || { tail -5 gpurun_out/tk3.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/tk3/run_kernel_trace.csv --steps 20 --marker tk_pass_a > gpurun_out/r6_topk_r50n_kernels.txt
rm -rf gpurun_out/tk3
true
