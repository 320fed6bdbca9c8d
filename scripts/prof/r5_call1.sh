# round 5 call 1: sanity bench, ResNet-50 serial-step profile (per grid), isolated per-layer table
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5c1_bench.json 2> gpurun_out/r5c1_bench.err
cat gpurun_out/r5c1_bench.json
timeout -k 10 300 python bench/r50_layers_f32.py > gpurun_out/r5c1_r50_layers.jsonl 2> gpurun_out/r5c1_r50_layers.err
tail -3 gpurun_out/r5c1_r50_layers.jsonl
PSX_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r50ser -o run -- python3 bench.py --model resnet50 --codec topk --steps 6 --warmup 3 --secondary none > gpurun_out/r5c1_r50ser.log 2>&1
python scripts/prof/kstats.py gpurun_out/r50ser/run_kernel_trace.csv --steps 5 > gpurun_out/r5c1_r50ser.txt
python scripts/prof/kstats.py gpurun_out/r50ser/run_kernel_trace.csv --steps 5 --grid "conv2_kernel|wgrad|wino|bn_|maxpool" > gpurun_out/r5c1_r50ser_grid.txt
head -30 gpurun_out/r5c1_r50ser.txt
rm -rf gpurun_out/r50ser
