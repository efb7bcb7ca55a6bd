# Pair-epilogue S stores through LDS (whole lines by consecutive lanes) against the DPP pair exchange (abl/base):
# the store-pattern microbenchmark, the pair / grid bit-identity tests + golden parity, then a same-box A/B at
# 64x40, 512x40 and 64x20. Repo root, GPU box.
set -e
O=gpurun_out/pair_store
mkdir -p $O
timeout -k 10 120 tools/store_cu_bench > $O/store_cu.txt 2>&1
grep -E "128 CUs|256 CUs| 64 CUs" $O/store_cu.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  > $O/tests.txt 2>&1 || { tail -n 30 $O/tests.txt; exit 1; }
tail -n 2 $O/tests.txt
bash tools/ab.sh ps64 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 40 --steps 20 | tee $O/ab64.txt
bash tools/ab.sh ps512 2 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 512 --n-atoms 40 --steps 10 | tee $O/ab512.txt
bash tools/ab.sh ps6420 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 20 --steps 30 | tee $O/ab6420.txt
