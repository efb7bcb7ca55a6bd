# A/B at the larger shapes: two launches (0) vs static pair grid (1), alternating
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/ab_grid2
mkdir -p $O
for cfg in "256 40" "512 40" "128 40"; do
  set -- $cfg
  for v in 0 1 0 1 0 1; do
    CHM_EDGE_PAIRS_LAYER=$v timeout -k 10 150 python bench.py --n-samples $1 --n-atoms $2 --steps 8 --warmup 3 \
      --no-cpu-baseline --no-api-legs --no-traffic > $O/b.json 2> $O/b.err
    python -c "import json;d=json.load(open('$O/b.json'));print('$1x$2 grid=$v', round(d['ms_per_step'],3), d['edge_events']['layer_repairs'])" | tee -a $O/summary.txt
  done
done
