# Round-2 closing measurements on the row-tile build: the GPU suite, then tools/r2_final.sh (rocprof
# kernel statistics + PMC traffic, default bench line, BASELINE configs, 2-rank rehearsal).
mkdir -p gpurun_out/v4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v4/gputests.txt 2>&1 || { tail -30 gpurun_out/v4/gputests.txt; exit 1; }
tail -2 gpurun_out/v4/gputests.txt
bash tools/r2_final.sh v4
