# round-5 reference measurements: default bench (PMC traffic, CPU baseline, API legs) + rocprof stats at 3 shapes
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/final5
mkdir -p $O
cd $R && timeout -k 10 420 python bench.py > $O/bench_default.json 2> $O/bench_default.err
cd /tmp && export TMPDIR=/tmp
for cfg in "512 40" "64 40" "64 20"; do
  set -- $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p$1x$2 -o run --output-format csv -- python3 $R/bench.py --n-samples $1 --n-atoms $2 --steps 5 --warmup 2 --no-cpu-baseline --no-api-legs --no-traffic > $O/bench_$1x$2.json 2> $O/bench_$1x$2.err
done
