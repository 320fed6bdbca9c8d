# pending GPU tests + stem reduce pre-sum A/B + step profile
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 240 $T tests/test_kernels_gpu.py tests/test_fp32_gpu.py > gpurun_out/t_kern_fp32.log 2>&1 || { tail -30 gpurun_out/t_kern_fp32.log; exit 1; }
tail -2 gpurun_out/t_kern_fp32.log
timeout -k 10 300 $T tests/test_native_loop_gpu.py tests/test_multirank_gpu.py > gpurun_out/t_multi.log 2>&1 || { tail -30 gpurun_out/t_multi.log; exit 1; }
tail -2 gpurun_out/t_multi.log
AB_CFGS="_ PSX_WGRAD_NO_PRESUM=1" bash scripts/prof/ab_env.sh || exit 1
bash scripts/prof/step_prof.sh
timeout -k 10 200 python bench/bgemm_f32.py > gpurun_out/bgemm.jsonl 2>&1 || { tail -5 gpurun_out/bgemm.jsonl; exit 1; }
cat gpurun_out/bgemm.jsonl
