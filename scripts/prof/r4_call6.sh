set -o pipefail
mkdir -p gpurun_out
AB_CFGS="PSX_WINO_WGF_MINHW=4 PSX_WINO_WGF_MINHW=8 PSX_WINO_WGF_MINHW=16" bash scripts/prof/ab_env.sh || exit 1
timeout -k 10 300 python bench.py --model resnet50 --codec topk --steps 10 --warmup 3 --secondary none > gpurun_out/r50.json 2>gpurun_out/r50.err || { tail -20 gpurun_out/r50.err; exit 1; }
cat gpurun_out/r50.json
bash scripts/prof/r50_prof.sh
