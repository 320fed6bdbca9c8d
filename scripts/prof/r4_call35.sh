# world-of-one in-process store: bench + transport tests, then the engine knob re-sweep
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_rccl_native_gpu.py tests/test_ps_gpu.py tests/test_native_loop_gpu.py tests/test_engine_gpu.py > gpurun_out/t_store.log 2>&1 || { tail -30 gpurun_out/t_store.log; exit 1; }
tail -1 gpurun_out/t_store.log
AB_CFGS="_ PSX_WGRAD_STREAM=1 PSX_WGRAD_RBATCH=0 PSX_WINO_WQ_MAX=16 PSX_WGRAD_NO_PRESUM=1 PSX_GRAPH_QUEUES=1" bash scripts/prof/ab_env.sh || exit 1
