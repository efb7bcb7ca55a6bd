# Round-2 closing measurements on the one-grid edge-layer build: the GPU suite, then tools/r2_final.sh (rocprof
# kernel statistics + PMC traffic, default bench line, BASELINE configs, 2-rank rehearsal).
mkdir -p gpurun_out/v5
true

bash tools/r2_final.sh v5
