# configs[4] (2048 ragged crystals of 1-80 atoms) as an 8-rank job: every rank's share run alone on this one GPU
# (bench.py --share 8 --share-rank r), so that the slowest rank, which sets the 8-GPU time, is known. Repo root,
# GPU box: bash tools/shares_ragged.sh <tag> [bench args]
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 300 python -u bench.py --ragged --n-samples 2048 --share 8 --share-rank $r --steps 10 --warmup 2 \
    --no-cpu-baseline --no-api-legs --no-traffic "$@" > $O/share8_r$r.json 2> $O/share8_r$r.err || { tail -n 20 $O/share8_r$r.err; exit 1; }
  echo "rank $r: $(python tools/bench_summary.py $O/share8_r$r.json | head -1)"
done
