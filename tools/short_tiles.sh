# Round 6, mixed row tiling (short last-round row tiles of edge layer 2): bit-identity tests, same-box A/B against
# the uniform tiling (CHM_EDGE_ROWS_SHORT=0) and the previous build (abl/base), bit-identity of whole steps against
# the previous build. Repo root, GPU box.
set -o pipefail
O=gpurun_out/short
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "short_row_tiles or trajectory_64x20 or staged_rows" > $O/tests.txt 2>&1 || { tail -n 40 $O/tests.txt; exit 1; }
tail -n 3 $O/tests.txt
bash tools/ab.sh s6420 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_EDGE_ROWS_SHORT=0" "CHM_X=0" -- \
  --n-samples 64 --n-atoms 20 --steps 40 || exit 1
bash tools/ab.sh s512 2 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 512 --steps 10 || exit 1
bash tools/ab.sh s64 2 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --steps 20 || exit 1
for n in "64 20" "64 40"; do
  set -- $n
  CHM_LIB=abl/base/libchemeleon_hip.so timeout -k 10 200 python tools/lib_diff.py run $O/base_$1x$2.npz --n-samples $1 --n-atoms $2 &&
    timeout -k 10 200 python tools/lib_diff.py run $O/new_$1x$2.npz --n-samples $1 --n-atoms $2 &&
    python tools/lib_diff.py compare $O/base_$1x$2.npz $O/new_$1x$2.npz || exit 1
done
