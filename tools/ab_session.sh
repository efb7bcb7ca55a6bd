# same-box A/B of a library build (repo root, GPU box): bit-identity of abl/$1 against the default build
# (seeded tools/lib_diff.py at 512x40 and 64x40), then tools/ab.sh at 512x40 and 64x40
set -o pipefail
export TMPDIR=/tmp
V=${1:-keep}
O=gpurun_out/abs_$V; mkdir -p $O
for n in 512 64; do
  timeout -k 10 300 python tools/lib_diff.py run $O/base$n.npz --n-samples $n > $O/libdiff_$n.txt 2>&1 || exit 1
  CHM_LIB=abl/$V/libchemeleon_hip.so timeout -k 10 300 python tools/lib_diff.py run $O/new$n.npz --n-samples $n >> $O/libdiff_$n.txt 2>&1 || exit 1
  python tools/lib_diff.py compare $O/new$n.npz $O/base$n.npz | tee -a $O/libdiff_$n.txt || exit 1
done
bash tools/ab.sh ${V}512 3 "CHM_X=0" "CHM_LIB=abl/$V/libchemeleon_hip.so" -- --steps 20 2>&1 | tee $O/ab512.txt
bash tools/ab.sh ${V}64 3 "CHM_X=0" "CHM_LIB=abl/$V/libchemeleon_hip.so" -- --steps 30 --n-samples 64 2>&1 | tee $O/ab64.txt
