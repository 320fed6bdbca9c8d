# round 5 call 5b: deterministic-mode slot spreading A/B + kernel split, merged PMC of the R50 1x1
# layers and the stem, and the README's stale rows (async N=1, staleness W=4/8, top-k N=1, R50 bf16)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_deterministic_gpu.py tests/test_fp32_gpu.py -k "determin or stem" > gpurun_out/r5c5_tests.log 2>&1 || { tail -40 gpurun_out/r5c5_tests.log; exit 1; }
tail -1 gpurun_out/r5c5_tests.log
ms() { grep -o '"ms_per_step": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
rm -f gpurun_out/r5c5_det_ab.jsonl
for rep in 1 2; do
for cfg in "0 " "1 det_slots=1" "1 det_slots=8" "1 det_slots=32"; do
  det=${cfg%% *}; tv=${cfg#* }
  for dt in fp32 bf16; do
    PSX_TUNE="$tv" PSX_DETERMINISTIC=$det timeout -k 10 200 python bench.py --steps 30 --warmup 10 --secondary none --dtype $dt > gpurun_out/det.json 2>gpurun_out/det.err || { tail -5 gpurun_out/det.err; exit 1; }
    echo "{\"dtype\": \"$dt\", \"deterministic\": $det, \"tune\": \"$tv\", \"rep\": $rep, \"ms_per_step\": $(ms gpurun_out/det.json)}" | tee -a gpurun_out/r5c5_det_ab.jsonl
  done
done
done
PSX_DETERMINISTIC=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/detk -o run -- python3 bench.py --steps 10 --warmup 5 --secondary none > gpurun_out/r5c5_detk.log 2>&1 || { tail -5 gpurun_out/r5c5_detk.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/detk/run_kernel_trace.csv --steps 10 > gpurun_out/r5c5_det_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ndetk -o run -- python3 bench.py --steps 10 --warmup 5 --secondary none > gpurun_out/r5c5_ndetk.log 2>&1 || { tail -5 gpurun_out/r5c5_ndetk.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/ndetk/run_kernel_trace.csv --steps 10 > gpurun_out/r5c5_nondet_kernels.txt
rm -rf gpurun_out/detk gpurun_out/ndetk
head -12 gpurun_out/r5c5_det_kernels.txt
for L in 64x256x56x1s1 256x64x56x1s1 1024x256x14x1s1 3x64x224x7s2; do
  ONLY=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc1_$L -o run -- python3 bench/r50_layers_f32.py > gpurun_out/pmc1_$L.log 2>&1 || { tail -5 gpurun_out/pmc1_$L.log; exit 1; }
  ONLY=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc2_$L -o run -- python3 bench/r50_layers_f32.py > gpurun_out/pmc2_$L.log 2>&1 || { tail -5 gpurun_out/pmc2_$L.log; exit 1; }
  ONLY=$L timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/pmc3_$L -o run -- python3 bench/r50_layers_f32.py > gpurun_out/pmc3_$L.log 2>&1 || { tail -5 gpurun_out/pmc3_$L.log; exit 1; }
  python3 scripts/prof/pmc_summary.py gpurun_out/pmc1_$L gpurun_out/pmc2_$L gpurun_out/pmc3_$L --top 4 --csv gpurun_out/r5c5_pmc_$L.csv > gpurun_out/r5c5_pmc_$L.txt
  rm -rf gpurun_out/pmc1_$L gpurun_out/pmc2_$L gpurun_out/pmc3_$L
  cat gpurun_out/r5c5_pmc_$L.txt
done
rm -f gpurun_out/r5c5_rows.jsonl
timeout -k 10 200 python bench.py --mode async --steps 30 --warmup 10 --secondary none > gpurun_out/rows.json 2>gpurun_out/rows.err || { tail -5 gpurun_out/rows.err; exit 1; }
echo "{\"row\": \"async N=1 fp32\", $(grep -o '"value": [0-9.]*' gpurun_out/rows.json), \"ms_per_step\": $(ms gpurun_out/rows.json)}" | tee -a gpurun_out/r5c5_rows.jsonl
timeout -k 10 200 python bench.py --codec topk --steps 30 --warmup 10 --secondary none > gpurun_out/rows.json 2>gpurun_out/rows.err || { tail -5 gpurun_out/rows.err; exit 1; }
echo "{\"row\": \"sync topk N=1 fp32\", $(grep -o '"value": [0-9.]*' gpurun_out/rows.json), \"ms_per_step\": $(ms gpurun_out/rows.json)}" | tee -a gpurun_out/r5c5_rows.jsonl
timeout -k 10 200 python bench.py --model resnet50 --codec topk --dtype bf16 --steps 10 --warmup 3 --secondary none > gpurun_out/rows.json 2>gpurun_out/rows.err || { tail -5 gpurun_out/rows.err; exit 1; }
echo "{\"row\": \"R50 topk N=1 bf16\", $(grep -o '"value": [0-9.]*' gpurun_out/rows.json), \"ms_per_step\": $(ms gpurun_out/rows.json)}" | tee -a gpurun_out/r5c5_rows.jsonl
timeout -k 10 300 python bench/async_staleness.py --workers 4 8 > gpurun_out/r5c5_staleness.jsonl 2>gpurun_out/r5c5_staleness.err || { tail -5 gpurun_out/r5c5_staleness.err; exit 1; }
cat gpurun_out/r5c5_staleness.jsonl
