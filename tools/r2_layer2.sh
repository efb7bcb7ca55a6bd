# k_edge16_layer (S exchanged through the XCD's L2, checked, repair launches) against the two-launch
# schedule, plus lags 6 and 16; preceded by the bit-identity tests.
O=gpurun_out/layer2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "row_tiles or tail_split" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
run() { local tag=$1 lay=$2 dbg=$3; shift 3
  CHM_EDGE_LAYER=$lay CHM_EDGE_DBG=$dbg timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  run 512_two_$rep 0 0 --steps 10 || exit 1
  
  run 512_layer_xcd_$rep 1 0 --steps 10 || exit 1
  run 64_two_$rep 0 0 --steps 20 --n-samples 64 || exit 1
  
  run 64_layer_xcd_$rep 1 0 --steps 20 --n-samples 64 || exit 1
done
for rep in 1 2; do
  CHM_EDGE_LAG=6 run 512_layer_lag6_$rep 1 0 --steps 10 || exit 1
  CHM_EDGE_LAG=16 run 512_layer_lag16_$rep 1 0 --steps 10 || exit 1
done
