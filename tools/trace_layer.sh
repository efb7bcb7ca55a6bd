# Block timeline of the one-grid edge kernel (k_edge16_layer) from one eager bench pass; repo root, GPU box.
# Usage: bash tools/trace_layer.sh <tag> <n_samples> [extra bench args]
O=gpurun_out/${1:-tlayer}; NS=${2:-512}; shift; shift
mkdir -p $O
CHM_EDGE_TRACE_LAYER=3 CHM_EDGE_TRACE=$O/t3.bin timeout -k 10 240 python bench.py --steps 1 --warmup 1 --no-graph \
  --no-cpu-baseline --no-api-legs --no-traffic --n-samples $NS "$@" > $O/b3.log 2>&1 || { tail -20 $O/b3.log; exit 1; }
python tools/trace_layer.py $O/t3.bin $NS 40
