# embed + the per-graph terms of edge layer 1 in one launch: the whole GPU suite, then a same-box A/B against the
# previous library at 64x20 and 64x40. Repo root, GPU box.
set -e
O=gpurun_out/embed_gb
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { tail -n 30 $O/gputests.txt; exit 1; }
tail -n 1 $O/gputests.txt
bash tools/ab.sh egb6420 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 20 --steps 30 | tee $O/ab6420.txt
bash tools/ab.sh egb64 2 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 40 --steps 20 | tee $O/ab64.txt
