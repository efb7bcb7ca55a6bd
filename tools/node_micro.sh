for M in 40960 5120; do
  for NK in "512 512" "1024 512" "512 1024"; do
    set -- $NK
    timeout -k 10 60 tools/gemm_bench $M $2 node $1 | grep -E "split16 k_node|blocks/CU" | head -3
  done
done
