# round 5 call 16: conv plan (fp32 power-of-two layers keep 64x128) step check; weight-gradient tile sweep
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c16.jsonl
for rep in 1 2; do
for tv in "" "cv_plan=r4"; do
  for args in "--dtype fp32" "--model resnet50 --codec topk --dtype fp32"; do
    st=30; case "$args" in *resnet50*) st=10;; esac
    PSX_TUNE="$tv" timeout -k 10 200 python bench.py $args --steps $st --warmup 3 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    echo "{\"tune\": \"$tv\", \"args\": \"$args\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c16.jsonl
  done
done
done
timeout -k 10 900 python bench/r50_wgrad_tiles.py > gpurun_out/r5c16_wtiles.jsonl 2>gpurun_out/r5c16_wtiles.err || { tail -5 gpurun_out/r5c16_wtiles.err; exit 1; }
cat gpurun_out/r5c16_wtiles.jsonl
