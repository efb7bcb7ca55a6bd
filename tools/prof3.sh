set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5k
for cfg in "512 40" "64 40" "64 20"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5k/p$1x$2 -o run --output-format csv -- python3 $R/bench.py --n-samples $1 --n-atoms $2 --steps 5 --warmup 2 --no-cpu-baseline --no-api-legs --no-traffic > $R/gpurun_out/r5k/bench_$1x$2.json 2> $R/gpurun_out/r5k/bench_$1x$2.err
done
