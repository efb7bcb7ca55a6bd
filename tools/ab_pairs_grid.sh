# A/B: edge layer 1 on pairs as two launches (CHM_EDGE_PAIRS_LAYER=0) vs both layers in one static grid (=1)
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/ab_grid
mkdir -p $O
for cfg in "64 20" "64 40" "512 40"; do
  set -- $cfg
  for v in 0 1 0 1; do
    CHM_EDGE_PAIRS_LAYER=$v timeout -k 10 150 python bench.py --n-samples $1 --n-atoms $2 --steps 10 --warmup 3 \
      --no-cpu-baseline --no-api-legs --no-traffic > $O/b_$1x$2_$v.json 2> $O/b_$1x$2_$v.err
    python -c "import json;d=json.load(open('$O/b_$1x$2_$v.json'));print('$1x$2 grid=$v', round(d['ms_per_step'],3), d['edge_events']['layer_repairs'], d['roofline']['avg_ms'])" | tee -a $O/summary.txt
  done
done
