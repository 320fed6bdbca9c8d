# round 5 call 13: R50 bf16 — conv LDS sized by the ring stages in use (A/B vs the full ring,
# variant ldsfull), deterministic cost, tile overrides; 1x1 layers vs hipBLASLt
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_conv_v2_gpu.py tests/test_kernels_gpu.py tests/test_fp32_gpu.py > gpurun_out/r5c13_t.log 2>&1 || { tail -40 gpurun_out/r5c13_t.log; exit 1; }
tail -1 gpurun_out/r5c13_t.log
timeout -k 10 300 python bench/r50_1x1_bf16.py > gpurun_out/r5c13_1x1.jsonl 2>gpurun_out/r5c13_1x1.err || { tail -5 gpurun_out/r5c13_1x1.err; exit 1; }
cat gpurun_out/r5c13_1x1.jsonl
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
V=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_ldsfull.so
rm -f gpurun_out/r5c13.jsonl
for rep in 1 2; do
for cfg in "default 1 " "ldsfull 1 " "default 0 " "default 1 cv_bm=64,cv_bn=64"; do
  set -- $cfg; lib=$1; det=$2; tv=${3:-}
  if [ $lib = ldsfull ]; then export PSX_KERNELS_LIB=$V; else unset PSX_KERNELS_LIB; fi
  for args in "--model resnet50 --codec topk --dtype bf16" "--model resnet50 --codec topk --dtype fp32" "--dtype bf16"; do
    st=10; case "$args" in *resnet50*) ;; *) st=30;; esac
    PSX_TUNE="$tv" PSX_DETERMINISTIC=$det timeout -k 10 200 python bench.py $args --steps $st --warmup 3 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    echo "{\"lib\": \"$lib\", \"det\": $det, \"tune\": \"$tv\", \"args\": \"$args\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c13.jsonl
  done
done
done
unset PSX_KERNELS_LIB
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b50k -o run -- python3 bench.py --model resnet50 --codec topk --dtype bf16 --steps 6 --warmup 3 --secondary none > gpurun_out/r5c13_b50k.log 2>&1 || { tail -5 gpurun_out/r5c13_b50k.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/b50k/run_kernel_trace.csv --steps 5 --grid "conv2_kernel|wgrad|bn_|stem" > gpurun_out/r5c13_r50_bf16_by_grid.txt
rm -rf gpurun_out/b50k
head -20 gpurun_out/r5c13_r50_bf16_by_grid.txt
