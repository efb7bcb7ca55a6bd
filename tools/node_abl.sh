# The split16 node GEMMs' K loops without their barrier / operand loads / A split (A/B builds -DCHM_NODE_ABL=n in
# abl/na<n>; wrong results), in cycles per kernel at 512x40 and 64x20. Repo root, GPU box: bash tools/node_abl.sh
O=$GRAFT_REPO_ROOT/gpurun_out/nabl; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for shape in "512 40" "64 20"; do
  set -- $shape
  for v in prod 1 2 4; do
    L=$GRAFT_REPO_ROOT/abl/na$v/libchemeleon_hip.so; [ $v = prod ] && L=$GRAFT_REPO_ROOT/chemeleon_amd/lib/libchemeleon_hip.so
    CHM_LIB=$L timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $O/v${v}_$1x$2 -o run --output-format csv \
      -- python3 $GRAFT_REPO_ROOT/bench.py --traffic-probe --n-samples $1 --n-atoms $2 > $O/v${v}_$1x$2.log 2>&1 || { tail -5 $O/v${v}_$1x$2.log; exit 1; }
    python3 $GRAFT_REPO_ROOT/tools/cycles_summary.py $O/v${v}_$1x$2 "$1x$2 $v" | grep node_gemm
  done
done
