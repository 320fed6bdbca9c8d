# round 5 call 24: are the 1x1 forward's BN sums atomic-throughput bound? det (2 x 64-bit atomics) vs
# float atomics, and 32 slot rows (variant s32) vs 8
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench/r50_1x1_bf16.py > gpurun_out/r5c24_1x1.jsonl 2>gpurun_out/r5c24_1x1.err || { tail -5 gpurun_out/r5c24_1x1.err; exit 1; }
cat gpurun_out/r5c24_1x1.jsonl
PSX_KERNELS_LIB=$GRAFT_REPO_ROOT/distributed-parameter-server-for-ml-training_amd/_native/variants/libpsx_kernels_s32.so timeout -k 10 300 python bench/r50_1x1_bf16.py > gpurun_out/r5c24_1x1_s32.jsonl 2>gpurun_out/r5c24_1x1_s32.err || { tail -5 gpurun_out/r5c24_1x1_s32.err; exit 1; }
cat gpurun_out/r5c24_1x1_s32.jsonl
