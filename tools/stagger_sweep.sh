# Edge-GEMM first-round stagger sweep (bench timing only). Run from the repo root on the GPU box.
mkdir -p gpurun_out/stg
for v in ${STG:-0 4 8 16}; do
  CHM_EDGE_STAGGER=$v timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/stg/s$v.log 2>&1 || exit 1
  echo "stagger $v: $(python tools/bench_summary.py gpurun_out/stg/s$v.log)"
done
