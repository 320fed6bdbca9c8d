# fused Winograd kernel: GPU tests, then the per-layer A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wino_fused_gpu.py -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wf_t.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/wf_t.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench/wino_fused_ab.py > gpurun_out/wf_ab.jsonl 2>&1 || { tail -20 gpurun_out/wf_ab.jsonl; exit 1; }
cat gpurun_out/wf_ab.jsonl
