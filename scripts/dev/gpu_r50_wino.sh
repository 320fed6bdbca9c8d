set -o pipefail
export TMPDIR=/tmp
for v in PSX_WINO=0 PSX_DUMMY=1 PSX_WINO_MAXHW=56; do
  env $v timeout -k 10 300 python bench.py --model resnet50 --codec topk --dtype fp32 --steps 10 --warmup 3 --secondary none > gpurun_out/r50_$v.log 2>&1 || { tail -20 gpurun_out/r50_$v.log; exit 3; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r50_$v.log | tr '\n' ' ' | sed "s/^/$v /"; echo
done
