# Round-2 closing measurements on the final round-2 build: the GPU suite, then tools/r2_final.sh (rocprof
# kernel statistics + PMC traffic, default bench line, BASELINE configs, 2-rank rehearsal).
mkdir -p gpurun_out/v7
true

bash tools/r2_final.sh v7
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v7/gputests.txt 2>&1; tail -2 gpurun_out/v7/gputests.txt
