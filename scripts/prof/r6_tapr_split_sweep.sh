# round 6: bf16 tap-reuse conv, pixel-tile width x split-K sweep per layer (bench/conv_layers.py)
mkdir -p gpurun_out/r6sw
for bn in 64 128 256; do
  for sp in 1 2 4 8; do
    export PSX_TUNE=cv_tapr_bn=$bn,cv_splits=$sp
    timeout -k 10 120 python bench/conv_layers.py > gpurun_out/r6sw/bn${bn}_sp${sp}.jsonl 2>/dev/null || exit 1
  done
done
