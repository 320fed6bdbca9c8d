# round 6 final numbers (same box): bench.py rows + kernel traces of the four step configs
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r6_final.jsonl
row() {  # name, bench args
  timeout -k 10 300 python bench.py "${@:2}" 2>/dev/null | grep '^{' | python -c "import json,sys; r=json.loads(sys.stdin.read()); r['row']='$1'; print(json.dumps(r))" >> gpurun_out/r6_final.jsonl || exit 1
}
row r18_fp32_default || exit 1
row r18_fp32_default_2 || exit 1
row r18_bf16 --dtype bf16 --secondary none || exit 1
row r18_fp32_topk --codec topk --secondary none || exit 1
row r18_fp32_async --mode async --secondary none || exit 1
row r50_fp32_topk --model resnet50 --codec topk --secondary none --steps 10 --warmup 3 || exit 1
row r50_bf16_topk --model resnet50 --codec topk --dtype bf16 --secondary none --steps 10 --warmup 3 || exit 1
bash scripts/prof/r6_fp32.sh || exit 1
