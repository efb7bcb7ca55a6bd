# bench with 1 / 2 / 3 stream lanes. Repo root, GPU box.
mkdir -p gpurun_out/lanes
for v in ${LANES:-1 2 3}; do
  timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --lanes $v "$@" > gpurun_out/lanes/b$v.log 2>&1 || { tail -n 20 gpurun_out/lanes/b$v.log; exit 1; }
  echo "lanes $v: $(python tools/bench_summary.py gpurun_out/lanes/b$v.log)"
done
