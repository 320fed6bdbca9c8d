# round 5 call 28: fused Winograd residual loads without a buffer descriptor (no scratch spills) —
# tests, same-box A/B vs variant wfbuf, then the full GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_wino_fused_gpu.py tests/test_wino_gpu.py > gpurun_out/r5c28_t.log 2>&1 || { tail -40 gpurun_out/r5c28_t.log; exit 1; }
tail -1 gpurun_out/r5c28_t.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
V=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_wfbuf.so
rm -f gpurun_out/r5c28.jsonl
for rep in 1 2 3; do
for lib in default wfbuf; do
  if [ $lib = wfbuf ]; then export PSX_KERNELS_LIB=$V; else unset PSX_KERNELS_LIB; fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  echo "{\"lib\": \"$lib\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c28.jsonl
done
done
unset PSX_KERNELS_LIB
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5c28_gpu.log 2>&1 || { tail -60 gpurun_out/r5c28_gpu.log; exit 1; }
tail -2 gpurun_out/r5c28_gpu.log
