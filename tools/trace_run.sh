# Block timelines of edge layer 1 (big and pp kernels, pp staggered). Repo root, GPU box.
mkdir -p gpurun_out/trace
for cfg in ${CFGS:-"0 0" "1 0" "1 8"}; do
  set -- $(echo $cfg | tr _ " ")
  CHM_EDGE_DBG=${DBG:-0} CHM_EDGE1_PP=$1 CHM_EDGE_STAGGER=${2:-0} CHM_EDGE_TRACE_LAYER=${LAYER:-1} CHM_EDGE_TRACE=gpurun_out/trace/t$1-$2.bin timeout -k 10 240 python bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline > gpurun_out/trace/b$1-$2.log 2>&1 || exit 1
  echo "== pp $1 stagger $2"; python tools/trace_summary.py gpurun_out/trace/t$1-$2.bin ${SUMARGS:-}
done
