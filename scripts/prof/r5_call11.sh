# round 5 call 11: pipelined conv epilogue (loads of a row chunk issued together) — conv tests, then
# same-box step A/B against the previous tree's kernels is not possible in one call: compare with
# r5_call8/9 numbers (same tree otherwise) + per-layer R50 fp32 isolated table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_conv_v2_gpu.py tests/test_kernels_gpu.py tests/test_fp32_gpu.py tests/test_wino_gpu.py tests/test_deterministic_gpu.py > gpurun_out/r5c11_t.log 2>&1 || { tail -40 gpurun_out/r5c11_t.log; exit 1; }
tail -1 gpurun_out/r5c11_t.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
for rep in 1 2; do
for args in "--dtype fp32" "--dtype bf16" "--model resnet50 --codec topk --dtype fp32" "--model resnet50 --codec topk --dtype bf16"; do
  st=30; case "$args" in *resnet50*) st=10;; esac
  timeout -k 10 200 python bench.py $args --steps $st --warmup 5 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  echo "{\"args\": \"$args\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c11_bench.jsonl
done
done
timeout -k 10 300 python bench/r50_layers_f32.py > gpurun_out/r5c11_r50_layers.jsonl 2> gpurun_out/r5c11_r50_layers.err || { tail -5 gpurun_out/r5c11_r50_layers.err; exit 1; }
tail -1 gpurun_out/r5c11_r50_layers.jsonl
