# A/B of the 16x16x32 edge kernels: microbenchmark, GPU parity suite (default = edge16), bench both ways.
O=gpurun_out/${1:-e16}
mkdir -p $O
timeout -k 10 120 tools/gemm_bench 819200 768 edgecmp > $O/gemm_l1.log 2>&1 && cat $O/gemm_l1.log &&
timeout -k 10 120 tools/gemm_bench 1638400 512 edgecmp > $O/gemm_l2.log 2>&1 && cat $O/gemm_l2.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${2:+-k "$2"} > $O/gputests.log 2>&1
rc=$?
tail -n 3 $O/gputests.log; grep -E "FAILED|Error" $O/gputests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
for e in 1 0 1 0; do
  CHM_EDGE16=$e timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-api-legs > $O/bench_e$e.log 2>&1 || { tail -n 30 $O/bench_e$e.log; exit 1; }
  echo "edge16=$e: $(python tools/bench_summary.py $O/bench_e$e.log)"
done
exit $rc
