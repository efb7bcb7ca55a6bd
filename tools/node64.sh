# 64x128 vs 64x64 split16 node-GEMM tiles on the short grids (M = P*N rows at 64x20, 64x40, 128x40)
set -e
O=${GRAFT_REPO_ROOT:-.}/gpurun_out/node64
mkdir -p $O
for M in 2560 5120 10240; do
  for NK in "512 512" "1024 512" "512 1024"; do
    set -- $NK
    timeout -k 10 60 tools/gemm_bench $M $2 node64 $1 >> $O/node64.txt 2>&1
  done
done
cat $O/node64.txt
