# fold probe, per-layer fused wgrad A/B + PMC, elastic sync tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/dev/fold_probe2.py || exit 1
Q="8,16,32,64" timeout -k 10 300 python bench/wino_wgrad_ab.py | tee gpurun_out/wgf_ab.jsonl || exit 1
bash scripts/prof/wgf_pmc.sh > gpurun_out/wgf_pmc.txt 2>&1; tail -30 gpurun_out/wgf_pmc.txt
timeout -k 10 200 python -u -m pytest tests/test_fp32_gpu.py -k engine_step -s -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/step_err.log 2>&1; grep -E "engine .*torch-fp32|passed|failed" gpurun_out/step_err.log | tail -70
timeout -k 10 900 python -u -m pytest tests/test_elastic_gpu.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/el.log 2>&1
rc=$?; tail -30 gpurun_out/el.log
exit $rc
