# 64-row S16 node GEMM, 16- vs 32-deep K-tiles, at the per-GPU shapes (M = 5120: 64x40; 10240: 128x40)
for M in 5120 10240 40960; do
  for NK in "512 512" "1024 512" "512 1024"; do
    set -- $NK
    timeout -k 10 60 tools/gemm_bench $M $2 node32 $1 || exit 1
  done
done
