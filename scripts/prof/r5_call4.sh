# round 5 call 4: deterministic (fixed-point) mode — tests + same-box cost A/B; PMC of R50 1x1 layers
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 200 $T tests/test_fp32_gpu.py -k stem > gpurun_out/r5c4_stem.log 2>&1 || { tail -40 gpurun_out/r5c4_stem.log; exit 1; }
tail -1 gpurun_out/r5c4_stem.log
ONLY=3x64x224x7s2 timeout -k 10 120 python bench/r50_layers_f32.py | tee gpurun_out/r5c4_stem.jsonl
timeout -k 10 700 $T tests/test_deterministic_gpu.py tests/test_wino_fused_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py > gpurun_out/r5c4_tests.log 2>&1 || { tail -40 gpurun_out/r5c4_tests.log; exit 1; }
tail -2 gpurun_out/r5c4_tests.log
rm -f gpurun_out/r5c4_det_ab.jsonl
for rep in 1 2; do
for dt in fp32 bf16; do
for det in 0 1; do
  PSX_DETERMINISTIC=$det timeout -k 10 200 python bench.py --steps 30 --warmup 10 --secondary none --dtype $dt > gpurun_out/det.json 2>gpurun_out/det.err || { tail -5 gpurun_out/det.err; exit 1; }
  echo "{\"dtype\": \"$dt\", \"deterministic\": $det, \"rep\": $rep, $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/det.json)}" | tee -a gpurun_out/r5c4_det_ab.jsonl
done
done
done
for L in 256x64x56x1s1 64x256x56x1s1 1024x256x14x1s1; do
  ONLY=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc1_$L -o run -- python3 bench/r50_layers_f32.py > gpurun_out/pmc1_$L.log 2>&1 || { tail -5 gpurun_out/pmc1_$L.log; exit 1; }
  ONLY=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc2_$L -o run -- python3 bench/r50_layers_f32.py > gpurun_out/pmc2_$L.log 2>&1 || { tail -5 gpurun_out/pmc2_$L.log; exit 1; }
  ONLY=$L timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/pmc3_$L -o run -- python3 bench/r50_layers_f32.py > gpurun_out/pmc3_$L.log 2>&1 || { tail -5 gpurun_out/pmc3_$L.log; exit 1; }
  python3 scripts/prof/pmc_summary.py gpurun_out/pmc1_$L --top 4 > gpurun_out/r5c4_pmc_$L.txt
  python3 scripts/prof/pmc_summary.py gpurun_out/pmc2_$L --top 4 >> gpurun_out/r5c4_pmc_$L.txt
  python3 scripts/prof/pmc_summary.py gpurun_out/pmc3_$L --top 4 >> gpurun_out/r5c4_pmc_$L.txt
  rm -rf gpurun_out/pmc1_$L gpurun_out/pmc2_$L gpurun_out/pmc3_$L
done
PSX_TUNE=wgrad_stream=0 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r50ser -o run -- python3 bench.py --model resnet50 --codec topk --steps 6 --warmup 3 --secondary none > gpurun_out/r5c4_r50ser.log 2>&1 || { tail -5 gpurun_out/r5c4_r50ser.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/r50ser/run_kernel_trace.csv --steps 5 > gpurun_out/r5c4_r50ser.txt
python scripts/prof/kstats.py gpurun_out/r50ser/run_kernel_trace.csv --steps 5 --grid "conv2_kernel|wgrad|wino|bn_|stem" > gpurun_out/r5c4_r50ser_grid.txt
head -25 gpurun_out/r5c4_r50ser.txt
rm -rf gpurun_out/r50ser
