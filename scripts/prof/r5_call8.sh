# round 5 call 8: deterministic mode as fixed-point slot pairs (no arrival / conversion tail):
# every deterministic-mode test, then the same-box cost A/B
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_bgemm_reg_gpu.py > gpurun_out/r5c8_bgemm_t.log 2>&1 || { tail -40 gpurun_out/r5c8_bgemm_t.log; exit 1; }
tail -1 gpurun_out/r5c8_bgemm_t.log
timeout -k 10 300 python bench/bgemm_f32.py > gpurun_out/r5c8_bgemm.jsonl 2>gpurun_out/r5c8_bgemm.err || { tail -5 gpurun_out/r5c8_bgemm.err; exit 1; }
cat gpurun_out/r5c8_bgemm.jsonl
timeout -k 10 900 $T tests/test_deterministic_gpu.py tests/test_wino_fused_gpu.py tests/test_fp32_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_conv_v2_gpu.py tests/test_wino_gpu.py > gpurun_out/r5c8_tests.log 2>&1 || { tail -40 gpurun_out/r5c8_tests.log; exit 1; }
tail -1 gpurun_out/r5c8_tests.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c8_det_ab.jsonl
for rep in 1 2; do
for dt in fp32 bf16; do
for det in 0 1; do
  PSX_DETERMINISTIC=$det timeout -k 10 200 python bench.py --steps 30 --warmup 10 --secondary none --dtype $dt > gpurun_out/det.json 2>gpurun_out/det.err || { tail -5 gpurun_out/det.err; exit 1; }
  echo "{\"dtype\": \"$dt\", \"deterministic\": $det, \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/det.json)}" | tee -a gpurun_out/r5c8_det_ab.jsonl
done
done
done
for det in 0 1; do
  PSX_DETERMINISTIC=$det timeout -k 10 200 python bench.py --model resnet50 --codec topk --steps 10 --warmup 3 --secondary none > gpurun_out/det.json 2>gpurun_out/det.err || { tail -5 gpurun_out/det.err; exit 1; }
  echo "{\"model\": \"resnet50\", \"dtype\": \"fp32\", \"deterministic\": $det, \"ms_per_step\": $(ms gpurun_out/det.json)}" | tee -a gpurun_out/r5c8_det_ab.jsonl
done
timeout -k 10 600 $T tests/test_multirank_gpu.py tests/test_elastic_gpu.py tests/test_native_loop_gpu.py > gpurun_out/r5c8_tests2.log 2>&1 || { tail -40 gpurun_out/r5c8_tests2.log; exit 1; }
tail -1 gpurun_out/r5c8_tests2.log
