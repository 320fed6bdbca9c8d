# round 5 call 21: full GPU suite on the current tree + step numbers (batched reduction with 8 loads
# in flight, bf16 ImageNet stem on the MFMA: A/B PSX_TUNE stem_direct=0)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_conv_v2_gpu.py -k stem7 -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c21_stem.log 2>&1 || { tail -40 gpurun_out/r5c21_stem.log; exit 1; }
tail -1 gpurun_out/r5c21_stem.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r5c21_gpu.log 2>&1 || { tail -60 gpurun_out/r5c21_gpu.log; exit 1; }
tail -2 gpurun_out/r5c21_gpu.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c21.jsonl
for tv in "" "stem_direct=0"; do
for args in "--dtype fp32" "--dtype bf16" "--model resnet50 --codec topk --dtype bf16" "--model resnet50 --codec topk --dtype fp32"; do
  st=30; case "$args" in *resnet50*) st=10;; esac
  case "$args$tv" in *stem_direct=0) case "$args" in *resnet50*bf16) ;; *) continue;; esac;; esac
  PSX_TUNE="$tv" timeout -k 10 200 python bench.py $args --steps $st --warmup 3 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  echo "{\"tune\": \"$tv\", \"args\": \"$args\", \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c21.jsonl
done
done
