# round 5 call 2: new RCCL world-1 p2p/abort/re-init test, elastic sha parity, bench secondaries
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 150 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_native_gpu.py::test_native_p2p_abort_reinit_world1 > gpurun_out/r5c2_rccl.log 2>&1 || { tail -30 gpurun_out/r5c2_rccl.log; exit 1; }
tail -3 gpurun_out/r5c2_rccl.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_elastic_gpu.py -k "scripted or (kill and 1-False)" > gpurun_out/r5c2_elastic.log 2>&1 || { tail -60 gpurun_out/r5c2_elastic.log; exit 1; }
tail -5 gpurun_out/r5c2_elastic.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5c2_bench.json 2> gpurun_out/r5c2_bench.err || { tail -20 gpurun_out/r5c2_bench.err; exit 1; }
cat gpurun_out/r5c2_bench.json
