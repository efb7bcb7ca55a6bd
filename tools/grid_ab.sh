# Pair-grid change: the grid tests, block timelines (traced build), then a same-box A/B against the committed
# library (abl/base) at 512x40 and 64x40. Repo root, GPU box.
set -e
O=gpurun_out/grid_ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "pairs_grid or pair_grid or golden or edge_pairs" > $O/tests.txt 2>&1 || { tail -n 30 $O/tests.txt; exit 1; }
tail -n 3 $O/tests.txt
for NA in "512 40" "64 40"; do
  set -- $NA
  CHM_LIB=abl/trace/libchemeleon_hip.so CHM_EDGE_TRACE=$O/grid_${1}x${2}.bin CHM_EDGE_TRACE_LAYER=4 \
    timeout -k 10 300 python bench.py --n-samples $1 --n-atoms $2 --steps 3 --warmup 1 --no-api-legs \
    --no-cpu-baseline --no-traffic > $O/t_${1}x${2}.json 2> $O/t_${1}x${2}.err
  python tools/grid_trace.py $O/grid_${1}x${2}.bin "${1}x${2}" | tee -a $O/trace_summary.txt
done
bash tools/ab.sh grid512 2 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 512 --n-atoms 40 --steps 10 | tee $O/ab512.txt
bash tools/ab.sh grid64 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 40 --steps 20 | tee $O/ab64.txt
