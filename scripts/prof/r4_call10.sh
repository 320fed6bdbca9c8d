# R50 fp32 weight-gradient shapes: timings per tile + PMC of the 56x56 256->64 1x1 layer
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/r50_wgrad_f32.py > gpurun_out/r50_wgrad.jsonl 2>&1 || { tail -5 gpurun_out/r50_wgrad.jsonl; exit 1; }
cat gpurun_out/r50_wgrad.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export ONE=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r50pmc1 -o run -- python3 bench/r50_wgrad_f32.py > gpurun_out/r50pmc1.log 2>&1 || { tail -5 gpurun_out/r50pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d gpurun_out/r50pmc2 -o run -- python3 bench/r50_wgrad_f32.py > gpurun_out/r50pmc2.log 2>&1 || { tail -5 gpurun_out/r50pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r50pmc3 -o run -- python3 bench/r50_wgrad_f32.py > gpurun_out/r50pmc3.log 2>&1 || { tail -5 gpurun_out/r50pmc3.log; exit 1; }
python3 scripts/prof/pmc_summary.py gpurun_out/r50pmc1 --top 3
python3 scripts/prof/pmc_summary.py gpurun_out/r50pmc2 --top 3
python3 scripts/prof/pmc_summary.py gpurun_out/r50pmc3 --top 3
