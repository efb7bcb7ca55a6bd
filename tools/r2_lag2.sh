# One-grid lag re-check on the final build: 8 / 10 / 12 at 512x40 and 64x40.
O=gpurun_out/lag2
mkdir -p $O
run() { local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  for L in 8 10 12; do CHM_EDGE_LAG=$L run 512_lag${L}_$rep --steps 10 || exit 1; done
  for L in 6 8 10; do CHM_EDGE_LAG=$L run 64_lag${L}_$rep --steps 30 --n-samples 64 || exit 1; done
done
