# round 5 call 18: where the bf16 1x1 forward's time goes (stats vs none; PMC of 64->256 @56)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench/r50_1x1_bf16.py > gpurun_out/r5c18_1x1.jsonl 2>gpurun_out/r5c18_1x1.err || { tail -5 gpurun_out/r5c18_1x1.err; exit 1; }
cat gpurun_out/r5c18_1x1.jsonl
L=64x256x56
ONLY=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc1 -o run -- python3 bench/r50_1x1_bf16.py > gpurun_out/pmc1.log 2>&1 || { tail -5 gpurun_out/pmc1.log; exit 1; }
ONLY=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc2 -o run -- python3 bench/r50_1x1_bf16.py > gpurun_out/pmc2.log 2>&1 || { tail -5 gpurun_out/pmc2.log; exit 1; }
ONLY=$L timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/pmc3 -o run -- python3 bench/r50_1x1_bf16.py > gpurun_out/pmc3.log 2>&1 || { tail -5 gpurun_out/pmc3.log; exit 1; }
ONLY=$L timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TA_BUSY_max GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc4 -o run -- python3 bench/r50_1x1_bf16.py > gpurun_out/pmc4.log 2>&1 || { tail -5 gpurun_out/pmc4.log; exit 1; }
python3 scripts/prof/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4 --top 6 --csv gpurun_out/r5c18_pmc.csv > gpurun_out/r5c18_pmc.txt
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4
cat gpurun_out/r5c18_pmc.txt
