# configs[4] ragged per-rank share (rank 0's Σn²-balanced 1/8 of 2048 crystals of 1-80 atoms) on the final tree
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/share5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 $R/bench.py --ragged --n-samples 2048 --share 8 --steps 5 --warmup 2 --no-cpu-baseline --no-api-legs --no-traffic > $O/bench_share8.json 2> $O/bench_share8.err
