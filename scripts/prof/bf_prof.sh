set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 0 1; do
PSX_WINO_BWDFOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bfp$f -o run -- python3 bench.py --steps 10 --warmup 5 --secondary none > gpurun_out/bfp$f.log 2>&1 || { tail -5 gpurun_out/bfp$f.log; exit 1; }
python scripts/prof/kstats.py gpurun_out/bfp$f/run_kernel_trace.csv --steps 8 > gpurun_out/bfp$f.txt
python scripts/prof/kstats.py gpurun_out/bfp$f/run_kernel_trace.csv --steps 8 --grid "wino|bn_bwd" > gpurun_out/bfp${f}_grid.txt
echo "== FOLD=$f"; head -1 gpurun_out/bfp$f.txt; grep -E "wino_fused|bn_bwd_apply|wino_dy" gpurun_out/bfp${f}_grid.txt | head -20
done
