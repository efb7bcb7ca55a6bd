# Edge-GEMM ablations inside the sampler (timing only; CHM_EDGE_DBG makes results wrong).
# Run from the repo root on the GPU box.
mkdir -p gpurun_out/abl
for d in ${ABL:-0 4 8 12 1}; do
  CHM_EDGE_DBG=$d timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl/d$d.json 2> gpurun_out/abl/d$d.err || exit 1
done
