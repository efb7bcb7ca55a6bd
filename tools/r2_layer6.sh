# One-grid A loads with the nt (streaming) hint: layer 2's S (CHM_EDGE_DBG=8192), layer 1's F (16384), both.
O=gpurun_out/layer6
mkdir -p $O
run() { local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  run 512_base_$rep --steps 10 || exit 1
  CHM_EDGE_DBG=8192 run 512_ntS_$rep --steps 10 || exit 1
  CHM_EDGE_DBG=16384 run 512_ntF_$rep --steps 10 || exit 1
  CHM_EDGE_DBG=24576 run 512_ntSF_$rep --steps 10 || exit 1
done
