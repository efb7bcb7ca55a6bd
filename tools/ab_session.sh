# same-box A/B (repo root, GPU box): the static one-grid map on a persistent grid (CHM_EDGE_DYN=3) against
# the dispatched static map (default below 1024 row tiles): bit-identity (seeded tools/lib_diff.py), then
# tools/ab.sh at the per-GPU shares 64x40 and 128x40
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/abs2; mkdir -p $O
for n in 64 128; do
  timeout -k 10 300 python tools/lib_diff.py run $O/base$n.npz --n-samples $n > $O/libdiff_$n.txt 2>&1 || exit 1
  CHM_EDGE_DYN=3 timeout -k 10 300 python tools/lib_diff.py run $O/new$n.npz --n-samples $n >> $O/libdiff_$n.txt 2>&1 || exit 1
  python tools/lib_diff.py compare $O/new$n.npz $O/base$n.npz | tee -a $O/libdiff_$n.txt || exit 1
done
bash tools/ab.sh pst64 3 "CHM_X=0" "CHM_EDGE_DYN=3" -- --steps 30 --n-samples 64 2>&1 | tee $O/ab64.txt
bash tools/ab.sh pst128 3 "CHM_X=0" "CHM_EDGE_DYN=3" -- --steps 20 --n-samples 128 2>&1 | tee $O/ab128.txt
