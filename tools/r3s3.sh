# r3 session 3: run-to-run determinism of the default build across processes, and which variant changes
# the result: default vs default, abl/s1 (half-line S stores) vs default, CHM_NODE_WIDE=1 vs default (64x40, 512x40)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s3; mkdir -p $O
run() { timeout -k 10 300 python tools/lib_diff.py run "$@" >> $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 1; }; }
for n in 64 512; do
  run $O/d1_$n.npz --n-samples $n
  run $O/d2_$n.npz --n-samples $n
  CHM_LIB=abl/s1/libchemeleon_hip.so run $O/s1_$n.npz --n-samples $n
  CHM_NODE_WIDE=1 run $O/w_$n.npz --n-samples $n
  for v in d2 s1 w; do echo "== $n: $v vs d1"; python tools/lib_diff.py compare $O/${v}_$n.npz $O/d1_$n.npz; done | tee -a $O/cmp.txt
done
# late job claim (abl/lc: -DCHM_LATE_CLAIM=1): bit-identity and same-box A/B at 512x40
CHM_LIB=abl/lc/libchemeleon_hip.so run $O/lc_512.npz --n-samples 512
echo "== 512: lc vs d1" | tee -a $O/cmp.txt; python tools/lib_diff.py compare $O/lc_512.npz $O/d1_512.npz | tee -a $O/cmp.txt
bash tools/ab.sh lc 3 "CHM_X=0" "CHM_LIB=abl/lc/libchemeleon_hip.so" -- --steps 20 2>&1 | tee $O/ab_lc.txt
