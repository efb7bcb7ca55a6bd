# split16 node GEMM 64-row tiles: microbenchmark (time vs K, 128-row tiles at 2/3 blocks per CU vs
# 64-row at 3/4, bit-identity) at M = 5120 .. 40960, the parity subset, and a same-box bench A/B
# at 64x40 and 256x40 (LIBS = previous and new library). Repo root, GPU box.
O=gpurun_out/${1:-node64}; mkdir -p $O
for M in 5120 10240 20480 40960; do
  timeout -k 10 90 tools/gemm_bench $M 1024 nodefix 512 >> $O/micro.log 2>&1 || { cat $O/micro.log; exit 1; }
done
cat $O/micro.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "teacher_forced or decoder_forward or shard or node" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -3 $O/parity.log
for shape in "--n-samples 64 --n-atoms 40" "--n-samples 256 --n-atoms 40"; do
  for rep in 1 2; do
    for l in ${LIBS}; do
      n=$(basename $l .so)
      CHM_LIB=$l timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $shape > $O/$n.log 2>&1 || exit 1
      echo "$shape $n: $(python tools/bench_summary.py $O/$n.log)" | tee -a $O/ab.txt
    done
  done
done
