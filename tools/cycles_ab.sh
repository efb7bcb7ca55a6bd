# Pair-grid cycles (GRBM_GUI_ACTIVE) at 512x40 of an A/B build (abl/<alt>) against the in-tree product, wall time aside:
# for timing-only ablation builds with wrong results. Repo root, GPU box: bash tools/cycles_ab.sh <tag> <alt> [dbg]
TAG=$1; ALT=$2; D=${3:-0}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in $ALT prod $ALT prod; do
  L=$GRAFT_REPO_ROOT/abl/$ALT/libchemeleon_hip.so; [ $v = prod ] && L=$GRAFT_REPO_ROOT/chemeleon_amd/lib/libchemeleon_hip.so
  rm -rf $O/$v
  CHM_LIB=$L CHM_EDGE_DBG=$D timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $O/$v -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --traffic-probe --n-samples 512 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  python3 $GRAFT_REPO_ROOT/tools/cycles_summary.py $O/$v "$v" | head -1
done
