# PMC of the stream-K GEMM
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/skpmc1 -o run -- python3 scripts/prof/sk_one.py > gpurun_out/skpmc1.log 2>&1 || { tail -5 gpurun_out/skpmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d gpurun_out/skpmc2 -o run -- python3 scripts/prof/sk_one.py > gpurun_out/skpmc2.log 2>&1 || { tail -5 gpurun_out/skpmc2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/skkt -o run -- python3 scripts/prof/sk_one.py > gpurun_out/skkt.log 2>&1 || { tail -5 gpurun_out/skkt.log; exit 1; }
python3 scripts/prof/pmc_summary.py gpurun_out/skpmc1 --top 8
python3 scripts/prof/pmc_summary.py gpurun_out/skpmc2 --top 8
grep -h "sk_gemm" gpurun_out/skkt/*kernel_stats.csv | head -3
