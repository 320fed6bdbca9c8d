set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3 4 5; do
for f in 0 1; do
  PSX_TAIL_SPLIT=$f timeout -k 10 200 python bench.py --steps 60 --warmup 10 --secondary none > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "TAIL=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
done
done
bash scripts/prof/step_prof.sh > /dev/null 2>&1 || { tail -5 gpurun_out/sprof.log; exit 1; }
head -1 gpurun_out/sprof.txt
