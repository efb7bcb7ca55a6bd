# Block timelines (CHM_EDGE_TRACE, s_memrealtime stamps) of edge layer 1 and 2 from one eager bench
# pass; repo root, GPU box. Usage: tools/trace_run.sh <tag> [bench args]
O=gpurun_out/${1:-trace}; shift
mkdir -p $O
for layer in 1 2; do
  CHM_EDGE_TRACE_LAYER=$layer CHM_EDGE_TRACE=$O/t$layer.bin timeout -k 10 240 python bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-api-legs "$@" > $O/b$layer.log 2>&1 || exit 1
  echo "== edge layer $layer"; python tools/trace_summary.py $O/t$layer.bin ${SUMARGS:-}
done
