# GPU suite on the final runtime, then one-grid S stores streaming (CHM_EDGE_DBG=1024) vs plain.
O=gpurun_out/layer4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { tail -30 $O/gputests.txt; exit 1; }
tail -2 $O/gputests.txt
run() { local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  run 512_plain_$rep --steps 10 || exit 1
  CHM_EDGE_DBG=1024 run 512_nt_$rep --steps 10 || exit 1
  run 64_plain_$rep --steps 20 --n-samples 64 || exit 1
  CHM_EDGE_DBG=1024 run 64_nt_$rep --steps 20 --n-samples 64 || exit 1
done
run 64x20 --steps 20 --n-samples 64 --n-atoms 20 || exit 1
