# One development iteration on the GPU box: parity suite, two bench lines, optional ablations.
# Usage: tools/r2_iter.sh <tag> [ablate]
O=gpurun_out/${1:-iter}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
tail -n 2 $O/gputests.log; grep -E "FAILED|Error|error" $O/gputests.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-api-legs > $O/bench$k.log 2>&1 || { tail -n 30 $O/bench$k.log; exit 1; }
  echo "bench $k: $(python tools/bench_summary.py $O/bench$k.log)"
done
if [ "$2" = "ablate" ]; then tools/r2_ablate.sh ${1:-iter}/abl; fi
