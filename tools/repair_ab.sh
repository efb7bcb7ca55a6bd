# One repair launch fewer per pair-grid layer: the grid tests (forced repairs bit-identical), then a same-box
# A/B against the previous library (abl/base) at 64x40 and 512x40. Repo root, GPU box.
set -e
O=gpurun_out/repair_ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "pairs_grid or pair_grid or repair" > $O/tests.txt 2>&1 || { tail -n 30 $O/tests.txt; exit 1; }
tail -n 3 $O/tests.txt
bash tools/ab.sh rep64 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 40 --steps 20 | tee $O/ab64.txt
bash tools/ab.sh rep512 2 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 512 --n-atoms 40 --steps 10 | tee $O/ab512.txt
