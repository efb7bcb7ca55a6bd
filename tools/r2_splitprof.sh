# rocprofv3 kernel stats of the 64x40 bench with and without the edge tail split. Repo root, GPU box.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/${1:-splitprof}; mkdir -p $O
for sp in 1 0; do
  CHM_EDGE_SPLIT=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s$sp -o run --output-format csv -- python3 $R/bench.py --n-samples ${NS:-64} --steps 5 --warmup 2 --no-cpu-baseline --no-api-legs > $O/s$sp.log 2>&1 || exit 1
done
