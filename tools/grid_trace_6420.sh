# Block timelines of the pair grid forced on at 64x20 (CHM_EDGE_LAYER_MIN=1; the default runs two launches there),
# lags 10 and 40. Repo root, GPU box.
set -e
O=gpurun_out/grid_trace_6420
mkdir -p $O
for LAG in 10 40; do
  CHM_LIB=abl/trace/libchemeleon_hip.so CHM_EDGE_LAYER_MIN=1 CHM_EDGE_LAG=$LAG CHM_EDGE_TRACE=$O/g_$LAG.bin CHM_EDGE_TRACE_LAYER=4 \
    timeout -k 10 300 python bench.py --n-samples 64 --n-atoms 20 --steps 3 --warmup 1 --no-api-legs \
    --no-cpu-baseline --no-traffic > $O/b_$LAG.json 2> $O/b_$LAG.err
  python tools/grid_trace.py $O/g_$LAG.bin "64x20 lag $LAG" | tee -a $O/summary.txt
  rm -f $O/g_$LAG.bin
done
