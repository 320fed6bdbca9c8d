# round 5 call 7: where deterministic mode's cost goes (probe knobs, wrong results) + det tests
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_deterministic_gpu.py tests/test_fp32_gpu.py -k "determin or stem" > gpurun_out/r5c7_tests.log 2>&1 || { tail -40 gpurun_out/r5c7_tests.log; exit 1; }
tail -1 gpurun_out/r5c7_tests.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c7_probe.jsonl
for cfg in "0 " "1 " "1 det_probe=1" "1 det_probe=2" "1 det_probe=3" "1 det_probe=4" "1 det_probe=5"; do
  det=${cfg%% *}; tv=${cfg#* }
  PSX_TUNE="$tv" PSX_DETERMINISTIC=$det timeout -k 10 200 python bench.py --steps 30 --warmup 10 --secondary none > gpurun_out/det.json 2>gpurun_out/det.err || { tail -5 gpurun_out/det.err; exit 1; }
  echo "{\"dtype\": \"fp32\", \"deterministic\": $det, \"tune\": \"$tv\", \"ms_per_step\": $(ms gpurun_out/det.json)}" | tee -a gpurun_out/r5c7_probe.jsonl
done
PSX_DETERMINISTIC=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/detk -o run -- python3 bench.py --steps 10 --warmup 5 --secondary none > gpurun_out/r5c7_detk.log 2>&1 || { tail -5 gpurun_out/r5c7_detk.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/detk/run_kernel_trace.csv --steps 10 > gpurun_out/r5c7_det_kernels.txt
rm -rf gpurun_out/detk
head -30 gpurun_out/r5c7_det_kernels.txt
