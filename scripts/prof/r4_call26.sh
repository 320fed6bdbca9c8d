set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_multirank_gpu.py -k "async_remote" > gpurun_out/t_async_q2.log 2>&1; echo "queues=2 rc=$?"; tail -3 gpurun_out/t_async_q2.log
PSX_GRAPH_QUEUES=0 timeout -k 10 500 $T tests/test_multirank_gpu.py -k "async_remote" > gpurun_out/t_async_q0.log 2>&1; echo "queues=default rc=$?"; tail -3 gpurun_out/t_async_q0.log
