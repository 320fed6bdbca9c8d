# full GPU suite + headline bench + ResNet-50 fused A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_$i.json 2>gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": 30, "warmup": 10, "ms_per_step": [0-9.]*' gpurun_out/bench_$i.json
grep -o '"bf16_compute": {[^}]*}' gpurun_out/bench_$i.json
done
for f in 1 0; do
PSX_WINO_FUSE=$f timeout -k 10 300 python bench.py --model resnet50 --codec topk --steps 10 --warmup 3 --secondary none > gpurun_out/r50_f$f.json 2>gpurun_out/r50.err || { tail -20 gpurun_out/r50.err; exit 1; }
echo "R50 fp32 topk FUSE=$f $(grep -o '"value": [0-9.]*' gpurun_out/r50_f$f.json) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r50_f$f.json)"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/gputests.log 2>&1
rc=$?
tail -6 gpurun_out/gputests.log
exit $rc
