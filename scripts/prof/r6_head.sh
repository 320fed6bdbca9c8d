# round 6: fused head with deeper load unrolls vs the base build (kernel trace of both + step A/B)
set -o pipefail
mkdir -p gpurun_out
BASE=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/libpsx_kernels_base.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp32_gpu.py -k "head or step" > gpurun_out/head_tests.log 2>&1 || { tail -30 gpurun_out/head_tests.log; exit 1; }
tail -1 gpurun_out/head_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for side in base new; do
  if [ $side = base ]; then export PSX_KERNELS_LIB=$BASE; else unset PSX_KERNELS_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/hd -o run -- python3 bench.py --steps 10 --warmup 5 --secondary none > gpurun_out/hd.log 2>&1 || { tail -5 gpurun_out/hd.log; exit 1; }
  python scripts/prof/kstats.py gpurun_out/hd/run_kernel_trace.csv --steps 8 > gpurun_out/head_$side.txt
  rm -rf gpurun_out/hd
done
unset PSX_KERNELS_LIB
bash scripts/prof/r6_ab.sh "PSX_KERNELS_LIB=$BASE" "PSX_X=1" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/head_ab_fp32.jsonl
