# One-grid job order A/B: [L1 L1 L2 L2 L2 L2] (default) vs [L1 L2 L2 L1 L2 L2] per row tile (CHM_EDGE_DBG=8192).
O=gpurun_out/layer5
mkdir -p $O
run() { local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "row_tiles" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
CHM_EDGE_DBG=8192 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "row_tiles" >> $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
grep passed $O/tests.txt
for rep in 1 2; do
  run 512_base_$rep --steps 10 || exit 1
  CHM_EDGE_DBG=8192 run 512_alt_$rep --steps 10 || exit 1
  run 64_base_$rep --steps 20 --n-samples 64 || exit 1
  CHM_EDGE_DBG=8192 run 64_alt_$rep --steps 20 --n-samples 64 || exit 1
done
