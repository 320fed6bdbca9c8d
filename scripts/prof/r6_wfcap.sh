# round 6: fp32 weight-gradient planners' split caps (PSX_AB_WFCAP wgrad2f, PSX_AB_W3FCAP wgrad3f) step A/B
set -o pipefail
mkdir -p gpurun_out
bash scripts/prof/r6_ab.sh "PSX_X=0" "PSX_AB_WFCAP=128" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wfcap_r18_wf128.jsonl
bash scripts/prof/r6_ab.sh "PSX_X=0" "PSX_AB_W3FCAP=256" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wfcap_r18_w3f256.jsonl
bash scripts/prof/r6_ab.sh "PSX_X=0" "PSX_AB_WFCAP=128" --model resnet50 --codec topk --steps 10 --warmup 3 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/wfcap_r50_wf128.jsonl
