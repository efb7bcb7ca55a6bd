# Round-2 final measurements (repo root, GPU box): rocprofv3 kernel stats at 512x40 and 64x40 with the
# PMC traffic passes (tools/r2_prof.sh), the default bench line (API legs + CPU baseline), the other
# BASELINE configs, and the 2-rank rehearsal of the multi-GPU path. Usage: tools/r2_final.sh <tag>
T=${1:-final}
O=gpurun_out/$T
bash tools/r2_prof.sh $T || exit 1
timeout -k 10 500 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
python tools/bench_summary.py $O/bench_default.log
timeout -k 10 200 python bench.py --n-samples 64 --n-atoms 20 --no-cpu-baseline --no-api-legs > $O/bench_64x20.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --n-samples 256 --n-atoms 40 --no-cpu-baseline --no-api-legs > $O/bench_256x40.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --n-samples 64 --n-atoms 40 --no-cpu-baseline --no-api-legs > $O/bench_64x40.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --ragged --n-samples 2048 --steps 3 --warmup 1 --no-cpu-baseline --no-api-legs > $O/bench_c4_2048.log 2>&1 || exit 1
for f in 64x20 256x40 64x40 c4_2048; do echo "$f $(python tools/bench_summary.py $O/bench_$f.log)"; done
bash tools/dist_rehearsal.sh && cp gpurun_out/dist_rehearsal.log $O/
