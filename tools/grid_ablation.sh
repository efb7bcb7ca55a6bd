# Pair grid (k_edge16_pairs_grid, the default schedule): launch time under CHM_EDGE_DBG ablations (profiling only,
# wrong results): 0 product, 4 no epilogue stores, 16 main loops only, 524288 pair P / Q rows not loaded,
# 4194304 pair jobs publish without waiting for their S stores (the drain). From r6 the epilogue bits (4, 524288) need
# an A/B build (CHM_BUILD_DEFS=-DCHM_PAIR_ABL=1, loaded with CHM_LIB), and wall times of data-changing variants carry a
# clock change: read them in cycles (tools/grid_ablation_cycles.sh). Repo root, GPU box:
#   bash tools/grid_ablation.sh <tag> [bench args]
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for d in ${GRID_DBG:-0 4 16 524288 4194304}; do
  CHM_EDGE_DBG=$d timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api-legs \
    --no-traffic "$@" > $O/grid_d$d.json 2> $O/grid_d$d.err || { tail -n 20 $O/grid_d$d.err; exit 1; }
  echo "dbg $d: $(python tools/bench_summary.py $O/grid_d$d.json | head -1)"
done
