# split16 node GEMM with the K loop split over 1 / 2 / 4 blocks per tile (tools/gemm_bench M K nodesplit N),
# at the per-GPU shares' node shapes (M = P * N: 64x20 2560, 64x40 5120, 128x40 10240, 512x40 40960)
for M in 2560 5120 10240 40960; do
  for KN in "512 512" "512 1024" "1024 512"; do
    set -- $KN
    timeout -k 10 60 tools/gemm_bench $M $1 nodesplit $2 || exit 1
  done
done
