# tail split: eager vs graph replay, and the graph's parallel-stream setting. Repo root, GPU box.
O=gpurun_out/${1:-split2}; mkdir -p $O
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --n-samples 64 --steps 6 --warmup 2 --no-cpu-baseline --no-api-legs $EXTRA > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"
}
for r in 1 2; do
  EXTRA=--no-graph run eager_s1_$r CHM_EDGE_SPLIT=1
  EXTRA=--no-graph run eager_s0_$r CHM_EDGE_SPLIT=0
  EXTRA= run graph_s1_$r CHM_EDGE_SPLIT=1
  EXTRA= run graph_s0_$r CHM_EDGE_SPLIT=0
  EXTRA= run graph_s1_q2_$r CHM_EDGE_SPLIT=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
  EXTRA= run graph_s1_q4_$r CHM_EDGE_SPLIT=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
done
