# deep-ring node GEMM variants against the default ring (tools/gemm_bench nodedeep)
for M in 2560 5120 40960; do
  for NK in "512 512" "1024 512" "512 1024"; do
    set -- $NK
    timeout -k 10 60 tools/gemm_bench $M $2 nodedeep $1
  done
done
