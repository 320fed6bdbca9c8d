# PMC counters of the fused Winograd weight gradient (scripts/prof/wgf_one.py), two passes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/gpmc1 -o run -- python3 scripts/prof/wgf_one.py > gpurun_out/gpmc1.log 2>&1 || { tail -5 gpurun_out/gpmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/gpmc2 -o run -- python3 scripts/prof/wgf_one.py > gpurun_out/gpmc2.log 2>&1 || { tail -5 gpurun_out/gpmc2.log; exit 1; }
python3 scripts/prof/pmc_summary.py gpurun_out/gpmc1 --top 5
python3 scripts/prof/pmc_summary.py gpurun_out/gpmc2 --top 5
