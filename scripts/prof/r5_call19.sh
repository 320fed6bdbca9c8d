# round 5 call 19: hardware bf16 conversion (v_cvt_pk_bf16_f32) vs the integer rounding (variant swbf16)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_kernels_gpu.py tests/test_conv_v2_gpu.py tests/test_engine_gpu.py tests/test_deterministic_gpu.py tests/test_weight_wire_gpu.py tests/test_wgrad_batch_gpu.py tests/test_resnet50_gpu.py > gpurun_out/r5c19_t.log 2>&1 || { tail -40 gpurun_out/r5c19_t.log; exit 1; }
tail -1 gpurun_out/r5c19_t.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
V=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_swbf16.so
rm -f gpurun_out/r5c19.jsonl
for rep in 1 2; do
for lib in default swbf16; do
  if [ $lib = swbf16 ]; then export PSX_KERNELS_LIB=$V; else unset PSX_KERNELS_LIB; fi
  for args in "--dtype bf16" "--model resnet50 --codec topk --dtype bf16"; do
    st=30; case "$args" in *resnet50*) st=10;; esac
    timeout -k 10 200 python bench.py $args --steps $st --warmup 3 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    echo "{\"lib\": \"$lib\", \"args\": \"$args\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c19.jsonl
  done
done
done
unset PSX_KERNELS_LIB
timeout -k 10 300 python bench/r50_1x1_bf16.py > gpurun_out/r5c19_1x1.jsonl 2>gpurun_out/r5c19_1x1.err || { tail -5 gpurun_out/r5c19_1x1.err; exit 1; }
cat gpurun_out/r5c19_1x1.jsonl
