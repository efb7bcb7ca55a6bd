# GPU parity tests + default bench (+ optional extra bench args) on the GPU box; run from the repo root.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -n 30 gpurun_out/gputests.log; exit 1; }
tail -n 2 gpurun_out/gputests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1 || { tail -n 30 gpurun_out/bench.log; exit 1; }
python tools/bench_summary.py gpurun_out/bench.log
