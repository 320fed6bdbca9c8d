# round 5 call 27: final tree — full GPU suite, smoke, bench.py (driver contract) with secondaries
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5c27_gpu.log 2>&1 || { tail -60 gpurun_out/r5c27_gpu.log; exit 1; }
tail -2 gpurun_out/r5c27_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5c27_smoke.log 2>&1 || { tail -20 gpurun_out/r5c27_smoke.log; exit 1; }
tail -1 gpurun_out/r5c27_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r5c27_bench.json 2>gpurun_out/r5c27_bench.err || { tail -5 gpurun_out/r5c27_bench.err; exit 1; }
grep '"metric"' gpurun_out/r5c27_bench.json
