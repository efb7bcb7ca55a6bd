# per-rank shares of the N = 1, 2, 4, 8 runs of the 512x40 headline, on one GPU (the ranks exchange nothing
# inside the timed region): n_samples 512 / N
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/${SHARES_TAG:-shares5}
mkdir -p $O
for rep in 1 2; do
  for n in 512 256 128 64; do
    timeout -k 10 200 python bench.py --n-samples $n --n-atoms 40 --steps 10 --warmup 3 --no-cpu-baseline --no-api-legs \
      --no-traffic > $O/b$n.json 2> $O/b$n.err
    python -c "import json;d=json.load(open('$O/b$n.json'));print('$n x40', round(d['ms_per_step'],3), round(d['value'],3), d['edge_events']['layer_repairs'])" | tee -a $O/summary.txt
  done
done
