# split16 node GEMM: time vs K at the 64x40 (M = 5120) and 512x40 (M = 40960) shapes (fixed cost = intercept),
# with / without the epilogue bias + SiLU and the A row scales; an empty launch for reference. Runs the
# current tools/gemm_bench and, when present, abl/gemm_bench_old (A/B). Repo root, GPU box.
O=gpurun_out/${1:-nodefix}; mkdir -p $O
for r in 1 2; do
  for bin in tools/gemm_bench abl/gemm_bench_old; do
    [ -x $bin ] || continue
    for M in 5120 40960; do
      echo "== $bin" >> $O/micro.log
      timeout -k 10 60 $bin $M 1024 nodefix 512 >> $O/micro.log 2>&1 || { cat $O/micro.log; exit 1; }
    done
  done
done
cat $O/micro.log
