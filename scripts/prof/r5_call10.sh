# round 5 call 10: Winograd GEMM reduction split (tests + A/B), bf16 step kernel profiles (R18, R50)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_wino_gpu.py -k "fwd or dgrad" > gpurun_out/r5c10_t.log 2>&1 || { tail -40 gpurun_out/r5c10_t.log; exit 1; }
tail -1 gpurun_out/r5c10_t.log
timeout -k 10 300 python bench/wino_split_ab.py > gpurun_out/r5c10_split.jsonl 2>gpurun_out/r5c10_split.err || { tail -5 gpurun_out/r5c10_split.err; exit 1; }
cat gpurun_out/r5c10_split.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bfk -o run -- python3 bench.py --dtype bf16 --steps 10 --warmup 5 --secondary none > gpurun_out/r5c10_bfk.log 2>&1 || { tail -5 gpurun_out/r5c10_bfk.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/bfk/run_kernel_trace.csv --steps 10 > gpurun_out/r5c10_bf16_kernels.txt
rm -rf gpurun_out/bfk
head -25 gpurun_out/r5c10_bf16_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b50k -o run -- python3 bench.py --model resnet50 --codec topk --dtype bf16 --steps 6 --warmup 3 --secondary none > gpurun_out/r5c10_b50k.log 2>&1 || { tail -5 gpurun_out/r5c10_b50k.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/b50k/run_kernel_trace.csv --steps 5 > gpurun_out/r5c10_r50_bf16_kernels.txt
python scripts/prof/kstats.py gpurun_out/b50k/run_kernel_trace.csv --steps 5 --grid "conv2_kernel|wgrad|bn_|stem" > gpurun_out/r5c10_r50_bf16_kernels_by_grid.txt
rm -rf gpurun_out/b50k
head -30 gpurun_out/r5c10_r50_bf16_kernels.txt
