# A/B of the node-GEMM tile order (CHM_NODE_LINEAR=1: launch order, 0: XCD-aware) and of both edge
# layers in one grid (k_edge16_layer, CHM_EDGE_LAYER=1, lag CHM_EDGE_LAG): bit-identity tests, then
# alternating bench runs at 512x40 and 64x40.
set -o pipefail
O=gpurun_out/layer1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "row_tiles or tail_split or at_size or decoder_forward" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
run() {  # $1 tag, $2 linear, $3 layer, $4 lag, rest: bench args
  local tag=$1 lin=$2 lay=$3 lag=$4; shift 4
  CHM_NODE_LINEAR=$lin CHM_EDGE_LAYER=$lay CHM_EDGE_LAG=$lag timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"
}
for rep in 1 2; do
  run 512_lin_$rep 1 0 10 --steps 10 || exit 1
  run 512_xcd_$rep 0 0 10 --steps 10 || exit 1
  run 512_layer10_$rep 0 1 10 --steps 10 || exit 1
  run 512_layer6_$rep 0 1 6 --steps 10 || exit 1
done
for rep in 1 2; do
  run 64_lin_$rep 1 0 10 --steps 20 --n-samples 64 || exit 1
  run 64_xcd_$rep 0 0 10 --steps 20 --n-samples 64 || exit 1
  run 64_layer10_$rep 0 1 10 --steps 20 --n-samples 64 || exit 1
  run 64_layer4_$rep 0 1 4 --steps 20 --n-samples 64 || exit 1
done
