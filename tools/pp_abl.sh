# Ablations of edge layer 1 on the pp kernel (timing only). Repo root, GPU box.
mkdir -p gpurun_out/ppabl
for d in ${ABL:-0 4 8 12}; do
  CHM_EDGE1_PP=${PP:-1} CHM_EDGE_DBG=$d timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ppabl/d$d.log 2>&1 || exit 1
  echo "pp ${PP:-1} dbg $d: $(python tools/bench_summary.py gpurun_out/ppabl/d$d.log)"
done
