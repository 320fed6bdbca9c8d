# round 5 call 12: same-box A/B of the pipelined conv epilogue (default) vs one row per round trip
# (variant library epi1, -D PSX_EPI_U=1)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
V=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_epi1.so
rm -f gpurun_out/r5c12_ab.jsonl
for rep in 1 2; do
for lib in default epi1; do
for args in "--dtype fp32" "--dtype bf16" "--model resnet50 --codec topk --dtype bf16" "--model resnet50 --codec topk --dtype fp32"; do
  st=30; case "$args" in *resnet50*) st=10;; esac
  if [ $lib = epi1 ]; then export PSX_KERNELS_LIB=$V; else unset PSX_KERNELS_LIB; fi
  timeout -k 10 200 python bench.py $args --steps $st --warmup 5 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
  echo "{\"lib\": \"$lib\", \"args\": \"$args\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c12_ab.jsonl
done
done
done
