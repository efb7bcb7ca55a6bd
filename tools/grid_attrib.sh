# Where a pair-grid job's time goes, in the grid (traced A/B build; CHM_EDGE_DBG ablations, wrong results):
# 0 product, 4 no pair-epilogue stores, 16 pair main loop only, 32768 F rows L2-resident, 65536 S rows L2-resident
# (layer-2 A operand), 98304 both. 512x40 and 64x40. Repo root, GPU box.
set -e
O=gpurun_out/grid_attrib
mkdir -p $O
for NA in "512 40" "64 40"; do
  set -- $NA
  for D in 0 4 16 32768 65536 98304; do
    CHM_LIB=abl/trace/libchemeleon_hip.so CHM_EDGE_DBG=$D CHM_EDGE_TRACE=$O/g_${1}_$D.bin CHM_EDGE_TRACE_LAYER=4 \
      timeout -k 10 300 python bench.py --n-samples $1 --n-atoms $2 --steps 2 --warmup 1 --no-api-legs \
      --no-cpu-baseline --no-traffic > $O/b_${1}_$D.json 2> $O/b_${1}_$D.err
    python tools/grid_trace.py $O/g_${1}_$D.bin "${1}x${2} dbg=$D" | tee -a $O/summary.txt
    rm -f $O/g_${1}_$D.bin
  done
done
