# HBM traffic of the dominant kernel (FETCH_SIZE and WRITE_SIZE in separate passes, as
# MI355X_MICROARCH.md prescribes), from a short bench run. Run from the repo root on the GPU box;
# then: python tools/traffic_summary.py gpurun_out/traffic > profiles/r1/traffic.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/traffic
mkdir -p $O
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-graph > $O/fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-graph > $O/write.log 2>&1
