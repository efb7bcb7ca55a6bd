# A/B: the decoder's independent kernels on one stream (CHM_DECODER_FORK=0) vs forked onto a second stream (=1)
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/ab_fork
mkdir -p $O
for cfg in "64 20" "64 40" "512 40"; do
  set -- $cfg
  for v in 0 1 0 1; do
    CHM_DECODER_FORK=$v timeout -k 10 150 python bench.py --n-samples $1 --n-atoms $2 --steps 10 --warmup 3 \
      --no-cpu-baseline --no-api-legs --no-traffic > $O/b.json 2> $O/b.err
    python -c "import json;d=json.load(open('$O/b.json'));print('$1x$2 fork=$v', round(d['ms_per_step'],3), d['edge_events']['layer_repairs'])" | tee -a $O/summary.txt
  done
done
