# Block timelines of one pair-grid launch (4th eager launch: bench.py's eager pass) at 512x40, 64x40, 256x40,
# traced build (abl/trace, CHM_BUILD_DEFS=-DCHM_GRID_TRACE=1). Repo root, GPU box.
set -e
O=gpurun_out/grid_trace
mkdir -p $O
for NA in "512 40" "64 40" "256 40"; do
  set -- $NA
  CHM_LIB=abl/trace/libchemeleon_hip.so CHM_EDGE_TRACE=$O/grid_${1}x${2}.bin CHM_EDGE_TRACE_LAYER=4 \
    timeout -k 10 300 python bench.py --n-samples $1 --n-atoms $2 --steps 3 --warmup 1 --no-api-legs \
    --no-cpu-baseline --no-traffic > $O/b_${1}x${2}.json 2> $O/b_${1}x${2}.err
  python tools/grid_trace.py $O/grid_${1}x${2}.bin "${1}x${2}" | tee -a $O/summary.txt
done
