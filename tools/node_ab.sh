# A/B of the node GEMM kernels (CHM_NODE_GLDS). Repo root, GPU box.
mkdir -p gpurun_out/node
for v in ${NV:-1 0}; do
  CHM_NODE_GLDS=$v timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/node/b$v.log 2>&1 || exit 1
  echo "node_glds $v: $(python tools/bench_summary.py gpurun_out/node/b$v.log)"
done
