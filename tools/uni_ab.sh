# Branch-free K loops (CHM_LOOP_UNI, edge16.hip) against the conditional form (abl/uni0): main-loop and whole-grid
# cycles, same-box bench A/B, whole steps bit-identical. Repo root, GPU box.
set -o pipefail
O=gpurun_out/uni; mkdir -p $O
for s in "512 40"; do
  set -- $s
  (cd /tmp && export TMPDIR=/tmp && for v in uni0 uni1; do
     L=$GRAFT_REPO_ROOT/abl/uni0/libchemeleon_hip.so; [ $v = uni1 ] && L=$GRAFT_REPO_ROOT/chemeleon_amd/lib/libchemeleon_hip.so
     for d in 16 0; do
       CHM_LIB=$L CHM_EDGE_DBG=$d timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/$O/${v}_d$d \
         -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --traffic-probe --n-samples $1 --n-atoms $2 \
         > $GRAFT_REPO_ROOT/$O/${v}_d$d.log 2>&1 || exit 1
       python3 $GRAFT_REPO_ROOT/tools/cycles_summary.py $GRAFT_REPO_ROOT/$O/${v}_d$d "$v dbg $d" | head -2
     done
   done) || exit 1
done
bash tools/ab.sh uni512 3 "CHM_LIB=abl/uni0/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 512 --steps 10 || exit 1
bash tools/ab.sh uni6420 3 "CHM_LIB=abl/uni0/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 20 --steps 40 || exit 1
bash tools/ab.sh uni64 2 "CHM_LIB=abl/uni0/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --steps 20 || exit 1
for n in "64 20" "64 40" "512 40"; do
  set -- $n
  CHM_LIB=abl/uni0/libchemeleon_hip.so timeout -k 10 200 python tools/lib_diff.py run $O/base_$1x$2.npz --n-samples $1 --n-atoms $2 &&
    timeout -k 10 200 python tools/lib_diff.py run $O/new_$1x$2.npz --n-samples $1 --n-atoms $2 &&
    python tools/lib_diff.py compare $O/base_$1x$2.npz $O/new_$1x$2.npz || exit 1
done
