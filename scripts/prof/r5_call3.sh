# round 5 call 3: partial-tile Winograd numerics + refactor checks, elastic parity, R50 per-layer + step A/B
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_wino_gpu.py tests/test_fp32_gpu.py tests/test_conv_v2_gpu.py > gpurun_out/r5c3_tests.log 2>&1 || { tail -40 gpurun_out/r5c3_tests.log; exit 1; }
tail -2 gpurun_out/r5c3_tests.log
timeout -k 10 400 $T tests/test_resnet50_gpu.py > gpurun_out/r5c3_r50t.log 2>&1 || { tail -40 gpurun_out/r5c3_r50t.log; exit 1; }
tail -2 gpurun_out/r5c3_r50t.log
timeout -k 10 300 python bench/r50_layers_f32.py > gpurun_out/r5c3_r50_layers.jsonl 2> gpurun_out/r5c3_r50_layers.err || { tail -5 gpurun_out/r5c3_r50_layers.err; exit 1; }
tail -1 gpurun_out/r5c3_r50_layers.jsonl
for v in "" "wino_maxhw=8" "wino_wgrad_maxhw=64"; do
  PSX_TUNE="$v" timeout -k 10 200 python bench.py --model resnet50 --codec topk --steps 10 --warmup 3 --secondary none > gpurun_out/r5c3_r50b.json 2>gpurun_out/r5c3_r50b.err || { tail -5 gpurun_out/r5c3_r50b.err; exit 1; }
  echo "tune=$v $(python -c "import json;r=json.load(open('gpurun_out/r5c3_r50b.json'));print(r['ms_per_step'], r['value'])")" | tee -a gpurun_out/r5c3_r50_ab.txt
done
timeout -k 10 700 $T tests/test_elastic_gpu.py -k "scripted" > gpurun_out/r5c3_elastic.log 2>&1 || { tail -30 gpurun_out/r5c3_elastic.log; exit 1; }
tail -2 gpurun_out/r5c3_elastic.log
