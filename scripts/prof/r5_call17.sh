# round 5 call 17: bf16 weight-gradient tile rule (64x128 up to 28x28) vs the cost model alone
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_conv_v2_gpu.py tests/test_wgrad_batch_gpu.py > gpurun_out/r5c17_t.log 2>&1 || { tail -40 gpurun_out/r5c17_t.log; exit 1; }
tail -1 gpurun_out/r5c17_t.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c17.jsonl
for rep in 1 2; do
for tv in "" "wg_plan=model"; do
  for args in "--dtype bf16" "--model resnet50 --codec topk --dtype bf16"; do
    st=30; case "$args" in *resnet50*) st=10;; esac
    PSX_TUNE="$tv" timeout -k 10 200 python bench.py $args --steps $st --warmup 3 --secondary none > gpurun_out/b.json 2>gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    echo "{\"tune\": \"$tv\", \"args\": \"$args\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/b.json)}" | tee -a gpurun_out/r5c17.jsonl
  done
done
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b50k -o run -- python3 bench.py --model resnet50 --codec topk --dtype bf16 --steps 6 --warmup 3 --secondary none > gpurun_out/r5c17_b50k.log 2>&1 || { tail -5 gpurun_out/r5c17_b50k.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/b50k/run_kernel_trace.csv --steps 5 > gpurun_out/r5c17_r50_bf16_kernels.txt
python scripts/prof/kstats.py gpurun_out/b50k/run_kernel_trace.csv --steps 5 --grid "conv2_kernel|wgrad|bn_|stem" > gpurun_out/r5c17_r50_bf16_by_grid.txt
rm -rf gpurun_out/b50k
head -30 gpurun_out/r5c17_r50_bf16_kernels.txt
