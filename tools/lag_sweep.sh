# the static pair grid's layer-2 lag (CHM_EDGE_LAG, pair tiles per XCD list) at 64x40 and 512x40
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/lag
mkdir -p $O
for cfg in "64 40" "512 40"; do
  set -- $cfg
  for lag in 10 3 6 16 10; do
    CHM_EDGE_LAG=$lag timeout -k 10 150 python bench.py --n-samples $1 --n-atoms $2 --steps 10 --warmup 3 \
      --no-cpu-baseline --no-api-legs --no-traffic > $O/b_$1x$2_$lag.json 2> $O/b_$1x$2_$lag.err
    python -c "import json;d=json.load(open('$O/b_$1x$2_$lag.json'));print('$1x$2 lag=$lag', round(d['ms_per_step'],3), d['edge_events']['layer_repairs'], d['roofline']['avg_ms'])" | tee -a $O/summary.txt
  done
done
