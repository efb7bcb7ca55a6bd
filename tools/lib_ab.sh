# A/B of two builds of the library in one GPU session: LIBS="path1 path2" (run from the repo root)
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for l in ${LIBS}; do
    n=$(basename $l .so)
    CHM_LIB=$l timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab/$n.log 2>&1 || exit 1
    echo "$n: $(python tools/bench_summary.py gpurun_out/ab/$n.log)"
  done
done
