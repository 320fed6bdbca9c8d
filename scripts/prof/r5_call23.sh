# round 5 call 23: ResNet-18 fp32 step knob re-check on the round-5 tree (deterministic default)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c23.jsonl
for rep in 1 2; do
for tv in "" "wgrad_stream=1" "wino_wgf_minhw=8" "wino_s2=1" "fin_grid=2048" "cv_plan=r4" "wino_wq_max=4" "tail_split=0"; do
  PSX_TUNE="$tv" timeout -k 10 200 python bench.py --steps 30 --warmup 5 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  echo "{\"tune\": \"$tv\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c23.jsonl
done
done
