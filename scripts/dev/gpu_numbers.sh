#!/bin/bash
# GPU-box helper: refresh the README performance table (one JSON line per run in gpurun_out/numbers.jsonl)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/numbers.jsonl
: > $OUT
run() {
  timeout -k 10 300 python bench.py "$@" > gpurun_out/num.log 2>&1 || { tail -20 gpurun_out/num.log; exit 3; }
  grep '"metric"' gpurun_out/num.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); r['args']=sys.argv[1:]; print(json.dumps(r))" "$@" >> $OUT
  echo "$* -> $(grep -o '"value": [0-9.]*' gpurun_out/num.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/num.log | head -1)"
}
run --secondary none
run --secondary none
run --dtype bf16 --secondary none
run --codec topk --secondary none
run --mode async --secondary none
run --model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3 --secondary none
run --model resnet50 --codec topk --steps 10 --warmup 3 --secondary none
