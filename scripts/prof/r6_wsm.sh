# round 6: bf16 weight-gradient planner, min pixel steps per split 8 -> 4 (PSX_AB_WSM) step A/B
set -o pipefail
mkdir -p gpurun_out
bash scripts/prof/r6_ab.sh "PSX_X=0" "PSX_AB_WSM=4" --dtype bf16 --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wsm_bf16.jsonl
bash scripts/prof/r6_ab.sh "PSX_X=0" "PSX_AB_WSM=4" --model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wsm_r50.jsonl
