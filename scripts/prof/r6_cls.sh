# round 6: stride-2 data-gradient parity-class dispatch order 3,2,1,0 vs 3,2,0,1 (PSX_AB_CLS)
set -o pipefail
mkdir -p gpurun_out
PSX_AB_CLS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_v2_gpu.py tests/test_fp32_gpu.py -k "dgrad or step" > gpurun_out/cls_tests.log 2>&1 || { tail -30 gpurun_out/cls_tests.log; exit 1; }
tail -1 gpurun_out/cls_tests.log
bash scripts/prof/r6_ab.sh "PSX_AB_CLS=0" "PSX_AB_CLS=1" --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/cls_fp32.jsonl
bash scripts/prof/r6_ab.sh "PSX_AB_CLS=0" "PSX_AB_CLS=1" --dtype bf16 --steps 30 --warmup 10 || exit 1
cp gpurun_out/ab.jsonl gpurun_out/cls_bf16.jsonl
