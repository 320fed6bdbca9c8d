set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/dev/numerics_probe.py "" nodet "wino=0" "wino_bnfold=0" "wino_bwdfold=0" "wino_wgf=0" "wino_fuse=0" "wino_maxhw=8" "wino_maxhw=16" "wino_wgrad=0" > gpurun_out/r5c5_numerics.jsonl 2> gpurun_out/r5c5_numerics.err || { tail -20 gpurun_out/r5c5_numerics.err; exit 1; }
cat gpurun_out/r5c5_numerics.jsonl
