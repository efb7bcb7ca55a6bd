# 64x20 (100 row tiles): two launches vs the pair grid at several lags
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/lag6420
mkdir -p $O
run() { timeout -k 10 120 env "$@" python bench.py --n-samples 64 --n-atoms 20 --steps 20 --warmup 3 --no-cpu-baseline --no-api-legs --no-traffic > $O/b.json 2> $O/b.err; python -c "import json;d=json.load(open('$O/b.json'));print('$*', round(d['ms_per_step'],3), d['edge_events']['layer_repairs'])" | tee -a $O/summary.txt; }
for rep in 1 2; do
  run CHM_EDGE_PAIRS_LAYER=0
  for lag in 1 2 4 10; do run CHM_EDGE_LAYER_MIN=64 CHM_EDGE_LAG=$lag; done
done
