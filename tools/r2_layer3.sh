# One-grid edge layers on by default: the whole GPU suite, then bench lines at lags 8 / 10 / 12 (512x40)
# and the 64x40 shard, plus the two-launch schedule for reference.
O=gpurun_out/layer3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { tail -30 $O/gputests.txt; exit 1; }
tail -2 $O/gputests.txt
run() { local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  CHM_EDGE_LAG=8 run 512_lag8_$rep --steps 10 || exit 1
  CHM_EDGE_LAG=10 run 512_lag10_$rep --steps 10 || exit 1
  CHM_EDGE_LAG=12 run 512_lag12_$rep --steps 10 || exit 1
  CHM_EDGE_LAYER=0 run 512_two_$rep --steps 10 || exit 1
done
for rep in 1 2; do
  CHM_EDGE_LAG=8 run 64_lag8_$rep --steps 20 --n-samples 64 || exit 1
  CHM_EDGE_LAG=10 run 64_lag10_$rep --steps 20 --n-samples 64 || exit 1
  CHM_EDGE_LAYER=0 run 64_two_$rep --steps 20 --n-samples 64 || exit 1
done
