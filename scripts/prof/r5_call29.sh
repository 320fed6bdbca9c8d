# round 5 call 29: final step numbers for the README (one box)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c29.jsonl
for args in "--dtype fp32" "--dtype bf16" "--model resnet50 --codec topk --dtype fp32" "--model resnet50 --codec topk --dtype bf16" "--codec topk --dtype fp32"; do
  st=30; case "$args" in *resnet50*) st=10;; esac
  timeout -k 10 200 python bench.py $args --steps $st --warmup 5 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  echo "{\"args\": \"$args\", \"ms_per_step\": $(ms gpurun_out/b.json), $(grep -o '"value": [0-9.]*' gpurun_out/b.json | head -1)}" | tee -a gpurun_out/r5c29.jsonl
done
