# r3 session 4: where the run-to-run difference of the sampling step comes from (tools/determinism.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s4; mkdir -p $O
for n in 64 512; do
  for r in a b; do
    timeout -k 10 300 python -u tools/determinism.py $O/det_${n}_$r.npz --n-samples $n 2>&1 | grep -v amdgpu.ids | tee -a $O/log.txt || exit 1
  done
  echo "== $n: cross-process" | tee -a $O/log.txt
  python tools/lib_diff.py compare $O/det_${n}_a.npz $O/det_${n}_b.npz | tee -a $O/log.txt
done
