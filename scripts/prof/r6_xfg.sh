# round 6: Winograd transform kernels' grid target (PSX_AB_XFG workgroups) step A/B
set -o pipefail
mkdir -p gpurun_out
bash scripts/prof/r6_ab.sh "PSX_AB_XFG=1024" "PSX_AB_XFG=512" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/xfg2_ab_1024_512.jsonl
bash scripts/prof/r6_ab.sh "PSX_AB_XFG=1024" "PSX_AB_XFG=256" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/xfg2_ab_1024_256.jsonl
bash scripts/prof/r6_ab.sh "PSX_AB_XFG=2048" "PSX_AB_XFG=1024" --model resnet50 --codec topk --steps 10 --warmup 3 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/xfg2_ab_r50.jsonl
