# Parity-mode noise under the captured step: the GPU suite, then the default bench line (API legs incl.
# sample() in both noise modes, CPU baseline skipped).
O=gpurun_out/tg
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { tail -30 $O/gputests.txt; exit 1; }
tail -2 $O/gputests.txt
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python tools/bench_summary.py $O/bench.log
tail -1 $O/bench.log | python -c "import json,sys; print(json.dumps(json.loads(sys.stdin.read())['api']))"
