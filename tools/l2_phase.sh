# Edge layer 2's epilogue phases (block timelines of the two-launch k_edge16<2, true>: main loop, SiLU pass (-> marker
# 4), half 0 (4 -> 5), half 1 (5 -> end)) with and without its agg stores (CHM_EDGE_DBG=4); repo root, GPU box.
O=gpurun_out/l2phase; mkdir -p $O
for d in ${DBGS:-0 4}; do
  CHM_EDGE_DBG=$d CHM_EDGE_PAIRS=0 CHM_EDGE_LAYER=0 CHM_EDGE_TRACE_LAYER=2 CHM_EDGE_TRACE=$O/t_$d.bin timeout -k 10 240 \
    python bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-api-legs --no-traffic "$@" > $O/b_$d.log 2>&1 ||
    { tail -20 $O/b_$d.log; exit 1; }
  echo "== dbg $d"; python tools/trace_summary.py $O/t_$d.bin ${SUMARGS:-}
done
