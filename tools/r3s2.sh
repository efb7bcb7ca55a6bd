# r3 session 2 A/B (repo root, GPU box): S half-line stores (abl/s1: -DCHM_S_HALF_LINES=1), + early job
# claim in the persistent edge kernel (abl/s1ec: + -DCHM_EARLY_CLAIM=1), node GEMM 128x256 tiles
# (CHM_NODE_WIDE=-1: by grid size) against the default build: bit-identity, same-box A/B, bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s2; mkdir -p $O
for n in 512 64; do
  CHM_NODE_WIDE=-1 CHM_LIB=abl/s1ec/libchemeleon_hip.so timeout -k 10 300 python tools/lib_diff.py run $O/new$n.npz --n-samples $n > $O/libdiff_$n.txt 2>&1 || { tail -20 $O/libdiff_$n.txt; exit 1; }
  timeout -k 10 300 python tools/lib_diff.py run $O/old$n.npz --n-samples $n >> $O/libdiff_$n.txt 2>&1 || { tail -20 $O/libdiff_$n.txt; exit 1; }
  python tools/lib_diff.py compare $O/new$n.npz $O/old$n.npz | tee -a $O/libdiff_$n.txt
done
bash tools/ab.sh s16 2 "CHM_X=0" "CHM_LIB=abl/s1/libchemeleon_hip.so" "CHM_LIB=abl/s1/libchemeleon_hip.so CHM_NODE_WIDE=-1" \
  "CHM_LIB=abl/s1ec/libchemeleon_hip.so CHM_NODE_WIDE=-1" -- --steps 20 2>&1 | tee $O/ab_s16.txt || exit 1
CHM_LIB=abl/s1ec/libchemeleon_hip.so CHM_NODE_WIDE=-1 bash tools/gpu_round.sh r3s2 bench:--steps=20
