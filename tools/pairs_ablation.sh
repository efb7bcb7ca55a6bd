# Edge layer 1 on pairs (k_edge16_pairs): where its time goes. CHM_EDGE_DBG (profiling only, wrong results):
# 0 = product, 16 = main loops only (both edge kernels), 4 = no epilogue stores, 131072 = no reverse-row
# stores, 262144 = reverse rows stored at the forward rows' places, 524288 = P / Q rows not loaded (zeros),
# 1048576 = P / Q rows read from global memory (not staged in LDS; exact), 2097152 = no exponent-byte stores (from r6
# the pair epilogue's bits 4, 131072, 262144, 524288, 2097152 need an A/B build, CHM_BUILD_DEFS=-DCHM_PAIR_ABL=1, loaded
# with CHM_LIB; and wall times of data-changing variants carry a clock change: tools/grid_ablation_cycles.sh). Runs the
# two-launch schedule (CHM_EDGE_PAIRS_LAYER=0) so that edge layer 1 has a launch of its own. Run from the repo root on
# the GPU box: bash tools/pairs_ablation.sh <tag> [bench args]
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for d in ${PAIRS_DBG:-0 16 4 131072 262144 524288 2097152}; do
  CHM_EDGE_PAIRS=1 CHM_EDGE_PAIRS_LAYER=0 CHM_EDGE_DBG=$d timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api-legs \
    --no-traffic "$@" > $O/pairs_d$d.json 2> $O/pairs_d$d.err || { tail -n 20 $O/pairs_d$d.err; exit 1; }
  python tools/bench_summary.py $O/pairs_d$d.json
done
