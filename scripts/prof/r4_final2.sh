# end-of-session check: full GPU suite + smoke + default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 || { tail -40 gpurun_out/full_gpu.log; exit 1; }
tail -1 gpurun_out/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -10 gpurun_out/bench_final.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_final.json | head -1
