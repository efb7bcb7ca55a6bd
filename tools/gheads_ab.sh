# k_graph_heads with its node-sum loads batched ahead of the adds (same order, so bit-identical by construction):
# the GPU parity suite, then a same-box A/B against the previous library. Repo root, GPU box.
set -e
O=gpurun_out/gheads
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { tail -n 30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
bash tools/ab.sh gh6420 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 20 --steps 30 | tee $O/ab6420.txt
bash tools/ab.sh gh64 2 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 40 --steps 20 | tee $O/ab64.txt
