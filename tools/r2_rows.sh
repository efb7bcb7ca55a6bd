set -o pipefail
mkdir -p gpurun_out/rt1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "row_tiles or tail_split or at_size or shard_invariance or graph_replay or decoder_forward" > gpurun_out/rt1/tests.txt 2>&1 || { tail -30 gpurun_out/rt1/tests.txt; exit 1; }
tail -3 gpurun_out/rt1/tests.txt
for r in 1 0 1 0; do CHM_EDGE_ROWS=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs --steps 10 > gpurun_out/rt1/b512_$r.log 2>&1 || exit 1; echo "512 rows=$r $(python tools/bench_summary.py gpurun_out/rt1/b512_$r.log)"; done
for r in 1 0 1 0; do CHM_EDGE_ROWS=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs --steps 20 --n-samples 64 > gpurun_out/rt1/b64_$r.log 2>&1 || exit 1; echo "64 rows=$r $(python tools/bench_summary.py gpurun_out/rt1/b64_$r.log)"; done
