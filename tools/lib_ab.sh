# Same-box A/B of an alternative build (abl/<alt>/libchemeleon_hip.so, CHM_BUILD_DEFS=... CHM_BUILD_LIB=...) against the
# in-tree product: pair-grid cycles (GRBM_GUI_ACTIVE) at 512x40, bench medians at 512x40 / 64x40 / 64x20, whole steps
# bit-identical at 64x20 and 512x40. Repo root, GPU box: bash tools/lib_ab.sh <tag> <alt>
set -o pipefail
TAG=$1; ALT=$2
O=gpurun_out/$TAG; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && for v in $ALT prod; do
   L=$GRAFT_REPO_ROOT/abl/$ALT/libchemeleon_hip.so; [ $v = prod ] && L=$GRAFT_REPO_ROOT/chemeleon_amd/lib/libchemeleon_hip.so
   CHM_LIB=$L timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/$O/$v -o run \
     --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --traffic-probe --n-samples 512 > $GRAFT_REPO_ROOT/$O/$v.log 2>&1 || exit 1
   python3 $GRAFT_REPO_ROOT/tools/cycles_summary.py $GRAFT_REPO_ROOT/$O/$v "$v" | head -1
 done) || exit 1
bash tools/ab.sh ${TAG}512 3 "CHM_LIB=abl/$ALT/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 512 --steps 10 || exit 1
bash tools/ab.sh ${TAG}64 2 "CHM_LIB=abl/$ALT/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --steps 20 || exit 1
bash tools/ab.sh ${TAG}6420 2 "CHM_LIB=abl/$ALT/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 20 --steps 40 || exit 1
for n in "64 20" "512 40"; do
  set -- $n
  CHM_LIB=abl/$ALT/libchemeleon_hip.so timeout -k 10 200 python tools/lib_diff.py run $O/alt_$1x$2.npz --n-samples $1 --n-atoms $2 &&
    timeout -k 10 200 python tools/lib_diff.py run $O/prod_$1x$2.npz --n-samples $1 --n-atoms $2 &&
    python tools/lib_diff.py compare $O/alt_$1x$2.npz $O/prod_$1x$2.npz || exit 1
done
