# The edge kernels' K loops without their synchronisation (A/B builds -DCHM_LOOP_ABL=n in abl/la<n>; wrong results),
# main loops only (CHM_EDGE_DBG=16), in cycles: what the per-K-tile barrier, the vmcnt / lgkmcnt waits and the loop's
# operand loads cost. One rocprofv3 pass (GRBM_GUI_ACTIVE + kernel trace) per variant; repo root, GPU box:
#   bash tools/loop_abl.sh <tag> [bench args]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in base ${LOOP_ABL:-1 2 4 8 15}; do
  if [ $v = base ]; then L=$R/chemeleon_amd/lib/libchemeleon_hip.so; else L=$R/abl/la$v/libchemeleon_hip.so; fi
  CHM_LIB=$L CHM_EDGE_DBG=${DBG:-16} timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $O/v$v -o run \
    --output-format csv -- python3 $R/bench.py --traffic-probe "$@" > $O/v$v.log 2>&1 || { echo "variant $v failed"; tail -5 $O/v$v.log; exit 1; }
  python3 $R/tools/cycles_summary.py $O/v$v "abl $v" | head -1
done
