set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py tests/test_native_loop_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?
tail -30 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
bash scripts/prof/det_ab.sh
