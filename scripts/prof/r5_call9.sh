# round 5 call 9: full GPU suite with deterministic mode as the default, smoke, bench (driver contract)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5c9_gpu.log 2>&1 || { tail -60 gpurun_out/r5c9_gpu.log; exit 1; }
tail -2 gpurun_out/r5c9_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
timeout -k 10 200 python bench.py > gpurun_out/r5c9_bench.json 2>gpurun_out/r5c9_bench.err || { tail -5 gpurun_out/r5c9_bench.err; exit 1; }
grep '"metric"' gpurun_out/r5c9_bench.json
