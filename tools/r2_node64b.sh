# Node GEMM launcher rule A/B (LIBS = previous and new library): kernel statistics of both builds at
# 256x40 (rocprofv3), then same-box bench lines at 64x40, 256x40 and 512x40. Repo root, GPU box.
O=gpurun_out/${1:-node64b}; mkdir -p $O
if [ -n "$PROF" ]; then
  for l in ${LIBS}; do
    n=$(basename $l .so)
    CHM_LIB=$GRAFT_REPO_ROOT/$l PROF_DIR=${1:-node64b}/prof_$n bash tools/rocprof_bench.sh --n-samples 256 --n-atoms 40 || exit 1
  done
fi
for shape in "--n-samples 64 --n-atoms 40" "--n-samples 256 --n-atoms 40" "--n-samples 512 --n-atoms 40"; do
  for rep in 1 2; do
    for l in ${LIBS}; do
      n=$(basename $l .so)
      CHM_LIB=$l timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $shape > $O/$n.log 2>&1 || exit 1
      echo "$shape $n: $(python tools/bench_summary.py $O/$n.log)" | tee -a $O/ab.txt
    done
  done
done
