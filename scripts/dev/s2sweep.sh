for cfg in "64 64 2" "64 128 2" "128 64 2" "128 128 2" "64 256 1" "64 128 1"; do
  set -- $cfg
  echo "BM=$1 BN=$2 WGM=$3"
  PSX_CV_BM=$1 PSX_CV_BN=$2 PSX_CV_WGM=$3 timeout -k 5 60 python bench/conv_probe.py 2,3,5,6,8,9 20 2>&1 | grep layer
done
