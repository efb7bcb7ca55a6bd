# A/B of environment settings on one box: tools/r2_ab.sh <tag> "ENV=a" "ENV=b" ... (interleaved, 2 rounds)
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
  k=0
  for e in "$@"; do
    k=$((k+1))
    env $e timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-api-legs > $O/ab$k-$r.log 2>&1 || { tail -n 20 $O/ab$k-$r.log; exit 1; }
    echo "$e (round $r): $(python tools/bench_summary.py $O/ab$k-$r.log)"
  done
done
