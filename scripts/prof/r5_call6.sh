# round 5 call 6: stem7 isolated; ResNet-50 fp32 step A/B (Winograd weight gradient on 56x56); R18 headline sanity
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ONLY=3x64x224x7s2 timeout -k 10 100 python bench/r50_layers_f32.py 2>/dev/null | head -1
for rep in 1 2; do
for v in "" "wino_wgrad_maxhw=64"; do
  PSX_TUNE="$v" timeout -k 10 200 python bench.py --model resnet50 --codec topk --steps 10 --warmup 3 --secondary none > gpurun_out/r5c6.json 2>gpurun_out/r5c6.err || { tail -5 gpurun_out/r5c6.err; exit 1; }
  echo "r50 tune=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5c6.json)" | tee -a gpurun_out/r5c6_ab.txt
done
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5c6_r18.json 2>gpurun_out/r5c6_r18.err || { tail -5 gpurun_out/r5c6_r18.err; exit 1; }
grep '"metric"' gpurun_out/r5c6_r18.json
