# Edge layer 2 without its SiLU-ablation select (abl/sel0, -DCHM_L2_SEL=0; the product from r6) against the build that
# keeps it (the product before; run with that build as 'prod'):
# whole-grid cycles, same-box bench A/B, whole steps bit-identical. Repo root, GPU box.
set -o pipefail
O=gpurun_out/sel; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && for v in sel0 prod; do
   L=$GRAFT_REPO_ROOT/abl/sel0/libchemeleon_hip.so; [ $v = prod ] && L=$GRAFT_REPO_ROOT/chemeleon_amd/lib/libchemeleon_hip.so
   CHM_LIB=$L timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/$O/$v -o run \
     --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --traffic-probe --n-samples 512 > $GRAFT_REPO_ROOT/$O/$v.log 2>&1 || exit 1
   python3 $GRAFT_REPO_ROOT/tools/cycles_summary.py $GRAFT_REPO_ROOT/$O/$v "$v" | head -1
 done) || exit 1
bash tools/ab.sh sel512 3 "CHM_LIB=abl/sel0/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 512 --steps 10 || exit 1
bash tools/ab.sh sel64 2 "CHM_LIB=abl/sel0/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --steps 20 || exit 1
bash tools/ab.sh sel6420 2 "CHM_LIB=abl/sel0/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 20 --steps 40 || exit 1
for n in "64 20" "512 40"; do
  set -- $n
  CHM_LIB=abl/sel0/libchemeleon_hip.so timeout -k 10 200 python tools/lib_diff.py run $O/base_$1x$2.npz --n-samples $1 --n-atoms $2 &&
    timeout -k 10 200 python tools/lib_diff.py run $O/new_$1x$2.npz --n-samples $1 --n-atoms $2 &&
    python tools/lib_diff.py compare $O/base_$1x$2.npz $O/new_$1x$2.npz || exit 1
done
