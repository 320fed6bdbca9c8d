# Same-box A/B of the fp32 headline step over Winograd switches (PSX_WINO_XF / PSX_WINO_FUSED),
# after the Winograd / fp32 / deterministic GPU tests; then a per-grid kernel profile.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_wino_gpu.py tests/test_fp32_gpu.py tests/test_deterministic_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wino_t.log 2>&1 || { tail -30 gpurun_out/wino_t.log; exit 1; }
tail -2 gpurun_out/wino_t.log
for rep in 1 2; do
for cfg in ${AB_CFGS:-"1 0" "0 0"}; do
  set -- $cfg
  PSX_WINO_XF=$1 PSX_WINO_FUSED=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 10 --secondary none > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  echo "XF=$1 FUSED=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wprof5 -o run -- python3 bench.py --steps 10 --warmup 5 --secondary none > gpurun_out/wprof5.log 2>&1
python scripts/prof/kstats.py gpurun_out/wprof5/run_kernel_trace.csv --steps 8 > gpurun_out/wprof5.txt
python scripts/prof/kstats.py gpurun_out/wprof5/run_kernel_trace.csv --steps 8 --grid "wino|conv2_kernel<float, 64, 64, 0, false, true|wgrad2f" > gpurun_out/wprof5_grid.txt
