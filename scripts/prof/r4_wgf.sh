# fused Winograd weight gradient: fold probe, engine numerics, same-box bench A/B, step profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/dev/fold_probe.py
timeout -k 10 600 python -u -m pytest tests/test_wino_wgrad_gpu.py tests/test_fp32_gpu.py tests/test_wino_fused_gpu.py tests/test_wino_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wgf_t2.log 2>&1
rc=$?; tail -8 gpurun_out/wgf_t2.log
AB_CFGS="PSX_WINO_WGF=0 PSX_WINO_WGF=1" bash scripts/prof/ab_env.sh || exit 1
bash scripts/prof/step_prof.sh
exit $rc
