# round 5 call 22: the multirank async tests alone (the full-suite run was killed for silence inside
# test_async_remote_workers[0-3-colocated]), verbose with per-test durations
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -k "async_remote_workers" -v --durations=0 --timeout 170 --timeout-method thread > gpurun_out/r5c22_mr.log 2>&1 || { tail -80 gpurun_out/r5c22_mr.log; exit 1; }
tail -30 gpurun_out/r5c22_mr.log
