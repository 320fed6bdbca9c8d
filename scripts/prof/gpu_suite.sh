set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
S0=$SECONDS; timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2>gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json; echo "bench_wall_s $((SECONDS - S0))"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/gputests.log 2>&1
rc=$?
tail -15 gpurun_out/gputests.log
exit $rc
