# the pair grid's per-call clears folded into the embedding launch: the whole GPU suite, then a same-box A/B against the
# previous library at 64x40 and 512x40. Repo root, GPU box.
set -e
O=gpurun_out/zero_gb
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { tail -n 30 $O/gputests.txt; exit 1; }
tail -n 1 $O/gputests.txt
bash tools/ab.sh zgb512 2 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 512 --n-atoms 40 --steps 10 | tee $O/ab512.txt
bash tools/ab.sh zgb64 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 40 --steps 20 | tee $O/ab64.txt
