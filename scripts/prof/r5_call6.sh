set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --model resnet50 --codec topk --steps 5 --warmup 2 --secondary none > gpurun_out/r5c6_r50.out 2> gpurun_out/r5c6_r50.err; echo "rc=$?"
tail -3 gpurun_out/r5c6_r50.out; tail -5 gpurun_out/r5c6_r50.err
ONLY=3x64x224x7s2 timeout -k 10 100 python bench/r50_layers_f32.py
