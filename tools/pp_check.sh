# A/B of the edge layer 1 kernels (CHM_EDGE1_PP) with parity tests on the pp kernel. Repo root, GPU box.
mkdir -p gpurun_out/pp
CHM_EDGE1_PP=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "split16 or cfg_pair or large or philox or graph" > gpurun_out/pp/tests.log 2>&1 || { tail -n 30 gpurun_out/pp/tests.log; exit 1; }
tail -n 1 gpurun_out/pp/tests.log
for v in ${PPV:-0 1}; do
  for st in ${STG:-0}; do
    CHM_EDGE1_PP=$v CHM_EDGE_STAGGER=$st timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/pp/b$v-$st.log 2>&1 || exit 1
    echo "pp $v stagger $st: $(python tools/bench_summary.py gpurun_out/pp/b$v-$st.log)"
  done
done
