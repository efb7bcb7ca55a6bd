# Edge layer 1 tail split (CHM_EDGE_SPLIT) A/B at 64x40, 256x40 and 512x40 (no split there), then the
# GPU suite. Repo root, GPU box. Usage: tools/r2_split.sh <tag>
O=gpurun_out/${1:-split}; mkdir -p $O
for sp in 1 0 1 0; do
  for n in 64 256 512; do
    CHM_EDGE_SPLIT=$sp timeout -k 10 200 python bench.py --n-samples $n --steps 6 --warmup 2 --no-cpu-baseline --no-api-legs > $O/b_${sp}_$n.log 2>&1 || { tail -5 $O/b_${sp}_$n.log; exit 1; }
    echo "split=$sp n=$n $(python tools/bench_summary.py $O/b_${sp}_$n.log)"
  done
done
