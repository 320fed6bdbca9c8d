# round 5 call 26: weight-gradient reduction chunks capped by loads per thread (A/B vs variant rcw)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_wgrad_batch_gpu.py tests/test_conv_v2_gpu.py -k "wgrad or reduce" > gpurun_out/r5c26_t.log 2>&1 || { tail -40 gpurun_out/r5c26_t.log; exit 1; }
tail -1 gpurun_out/r5c26_t.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
V=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_rcw.so
rm -f gpurun_out/r5c26.jsonl
for rep in 1 2; do
for lib in default rcw; do
  if [ $lib = rcw ]; then export PSX_KERNELS_LIB=$V; else unset PSX_KERNELS_LIB; fi
  for args in "--dtype bf16" "--dtype fp32" "--model resnet50 --codec topk --dtype bf16"; do
    st=30; case "$args" in *resnet50*) st=10;; esac
    timeout -k 10 200 python bench.py $args --steps $st --warmup 3 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    echo "{\"lib\": \"$lib\", \"args\": \"$args\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c26.jsonl
  done
done
done
