# round 6: bf16 tap-reuse conv per layer (bench/conv_layers.py) at each pixel-tile width
mkdir -p gpurun_out
for bn in default 64 128 256; do
  if [ $bn = default ]; then unset PSX_TUNE; else export PSX_TUNE=cv_tapr_bn=$bn; fi
  timeout -k 10 120 python bench/conv_layers.py > gpurun_out/r6_tapr_$bn.jsonl 2>gpurun_out/r6_tapr_$bn.err || exit 1
done
