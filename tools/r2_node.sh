# split16 node GEMM, K-interleave 1 vs 2 wave groups (tools/gemm_bench nodeks) at the 64x40 (M = 5120)
# and 512x40 (M = 40960) node shapes, then the bench at both sizes with CHM_NODE_KS=1 / 2. Repo root, GPU box.
O=gpurun_out/${1:-node}; mkdir -p $O
for M in 5120 40960; do
  for NK in "512 512" "512 1024" "1024 512"; do
    set -- $NK
    timeout -k 10 60 tools/gemm_bench $M $2 nodeks $1 >> $O/micro.log 2>&1 || { cat $O/micro.log; exit 1; }
  done
done
cat $O/micro.log
for ks in 1 2 1 2; do
  for n in 64 512; do
    CHM_NODE_KS=$ks timeout -k 10 200 python bench.py --n-samples $n --steps 5 --warmup 2 --no-cpu-baseline --no-api-legs > $O/b_${ks}_$n.log 2>&1 || { tail -5 $O/b_${ks}_$n.log; exit 1; }
    echo "KS=$ks n=$n $(python tools/bench_summary.py $O/b_${ks}_$n.log)"
  done
done
