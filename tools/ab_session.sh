# same-box A/B of library builds (repo root, GPU box): bit-identity of the default build against abl/base
# (tools/lib_diff.py, seeded), then tools/ab.sh over the builds at 512x40 and 64x40
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/abs; mkdir -p $O
for n in 512 64; do
  CHM_LIB=abl/base/libchemeleon_hip.so timeout -k 10 300 python tools/lib_diff.py run $O/base$n.npz --n-samples $n > $O/libdiff_$n.txt 2>&1 || exit 1
  timeout -k 10 300 python tools/lib_diff.py run $O/new$n.npz --n-samples $n >> $O/libdiff_$n.txt 2>&1 || exit 1
  python tools/lib_diff.py compare $O/new$n.npz $O/base$n.npz | tee -a $O/libdiff_$n.txt || exit 1
done
bash tools/ab.sh segtab 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_LIB=abl/l1/libchemeleon_hip.so" "CHM_X=0" -- --steps 20 2>&1 | tee $O/ab512.txt
bash tools/ab.sh segtab64 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --steps 30 --n-samples 64 2>&1 | tee $O/ab64.txt
