# Edge layer 2 (k_edge16<EPI_SEGMEAN>, two-launch schedule) at 512x40: where its tile time goes. CHM_EDGE_DBG
# (profiling only, wrong results): 0 product, 16 main loop only, 8 no SiLU, 32 no segment sums, 4 no agg stores
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/l2abl
mkdir -p $O
for d in 0 16 8 32 4 40 0; do
  CHM_EDGE_PAIRS_LAYER=0 CHM_EDGE_DBG=$d timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api-legs \
    --no-traffic > $O/d$d.json 2> $O/d$d.err
  python -c "import json;d=json.load(open('$O/d$d.json'));print('dbg $d', 'L2 %.3f ms' % d['edge_layer2']['avg_ms'], 'L1 %.3f ms' % d['edge_layer1']['avg_ms'], 'step %.2f' % d['ms_per_step'])" | tee -a $O/summary.txt
done
