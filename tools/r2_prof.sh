# rocprofv3 kernel statistics (512x40 and the 8-GPU per-rank share 64x40) and the PMC traffic passes
# of the current default build; run from the repo root on the GPU box. Usage: tools/r2_prof.sh <tag>
T=${1:-prof}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s512 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api-legs > $O/s512.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s64 -o run --output-format csv -- python3 $R/bench.py --n-samples 64 --steps 5 --warmup 2 --no-cpu-baseline --no-api-legs > $O/s64.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/traffic/fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-api-legs --no-graph > $O/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/traffic/write -o write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-api-legs --no-graph > $O/write.log 2>&1 || exit 1
cd $R && python tools/traffic_summary.py $O/traffic > $O/traffic.json && tail -n 1 $O/s512.log && tail -n 1 $O/s64.log
