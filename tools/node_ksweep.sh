# Node GEMM (split16, default tiling) time against K at the short-grid shapes: the fixed cost of a launch
# against the per-K-step cost (tools/gemm_bench nodedeep; first line of each run = the default ring).
for M in 2560 5120 40960; do
  for K in 64 128 256 512 1024; do
    timeout -k 10 60 tools/gemm_bench $M 512 nodedeep $K | head -n 1
  done
done
