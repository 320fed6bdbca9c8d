# round 5 call 15: the round-5 conv tile plan vs round 4's (PSX_TUNE cv_plan=r4), both models, both dtypes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_conv_v2_gpu.py tests/test_kernels_gpu.py tests/test_fp32_gpu.py tests/test_resnet50_gpu.py > gpurun_out/r5c15_t.log 2>&1 || { tail -40 gpurun_out/r5c15_t.log; exit 1; }
tail -1 gpurun_out/r5c15_t.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c15.jsonl
for rep in 1 2; do
for tv in "" "cv_plan=r4"; do
  for args in "--dtype fp32" "--dtype bf16" "--model resnet50 --codec topk --dtype bf16" "--model resnet50 --codec topk --dtype fp32"; do
    st=30; case "$args" in *resnet50*) st=10;; esac
    PSX_TUNE="$tv" timeout -k 10 200 python bench.py $args --steps $st --warmup 3 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    echo "{\"tune\": \"$tv\", \"args\": \"$args\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c15.jsonl
  done
done
done
