# Edge-kernel epilogue ablations (CHM_EDGE_DBG bits, wrong results, timing only): per-kernel HIP-event
# times from bench.py. Run from the repo root on the GPU box. Usage: tools/r2_ablate.sh <tag> [bench args]
O=gpurun_out/${1:-abl}; shift
mkdir -p $O
for d in 0 16 4 8 32 40 0; do
  CHM_EDGE_DBG=$d timeout -k 10 200 python -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-api-legs "$@" > $O/d$d.log 2>&1 || { tail -n 20 $O/d$d.log; exit 1; }
  echo "dbg=$d: $(python tools/bench_summary.py $O/d$d.log)"
done
