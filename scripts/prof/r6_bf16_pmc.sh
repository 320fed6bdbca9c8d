# round 6: PMC counters of the bf16 ResNet-18 step (two passes, counters in their own runs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
export PSX_TUNE=wgrad_stream=0
timeout -s KILL 240 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/r6pmc1 -o run -- python3 bench.py --dtype bf16 --steps 3 --warmup 2 --secondary none > gpurun_out/r6pmc1.log 2>&1 || { tail -5 gpurun_out/r6pmc1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/r6pmc2 -o run -- python3 bench.py --dtype bf16 --steps 3 --warmup 2 --secondary none > gpurun_out/r6pmc2.log 2>&1 || { tail -5 gpurun_out/r6pmc2.log; exit 1; }
python scripts/prof/pmc_summary.py gpurun_out/r6pmc1 gpurun_out/r6pmc2 --top 40 --csv gpurun_out/r6_bf16_pmc.csv > gpurun_out/r6_bf16_pmc.txt 2>&1
rm -rf gpurun_out/r6pmc1 gpurun_out/r6pmc2
