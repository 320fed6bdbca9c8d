# round 5 call 14: conv tile sweep on ResNet-50's 1x1 / strided layers (bf16, fp32)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python bench/r50_tiles.py > gpurun_out/r5c14_tiles.jsonl 2>gpurun_out/r5c14_tiles.err || { tail -5 gpurun_out/r5c14_tiles.err; exit 1; }
cat gpurun_out/r5c14_tiles.jsonl
