# GPU test suite + default bench (API legs and CPU baseline included); run from the repo root on the GPU box.
# Usage: tools/r2_check.sh <out-subdir> [pytest -k expression]
O=gpurun_out/${1:-check}
mkdir -p $O
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${2:+-k "$2"} > $O/gputests.log 2>&1
rc=$?
tail -n 5 $O/gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -n 30 $O/bench.log; exit 1; }
python tools/bench_summary.py $O/bench.log
exit $rc
