# A/B of two environment settings on bench.py, interleaved, same box: r6_ab.sh "ENV_A" "ENV_B" bench-args...
A="$1"; B="$2"; shift 2
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for rep in 1 2 3; do
  for side in A B; do
    if [ $side = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 200 python bench.py --secondary none "$@" 2>/dev/null | grep '^{' | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'side': '$side', 'env': '$E', 'rep': $rep, 'ms': r['ms_per_step']}))" >> gpurun_out/ab.jsonl || exit 1
  done
done
