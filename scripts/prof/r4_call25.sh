# rest of the GPU suite (multirank + elastic), smoke, bench
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 400 --timeout-method thread"
timeout -k 10 1000 $T tests/test_multirank_gpu.py tests/test_elastic_gpu.py > gpurun_out/t_full.log 2>&1 || { tail -40 gpurun_out/t_full.log; exit 1; }
tail -3 gpurun_out/t_full.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2>gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
