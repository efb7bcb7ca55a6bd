# Repair-launch grid size (CHM_REPAIR_GRID) A/B: their no-op cost per launch at 64x40 and 512x40.
O=gpurun_out/repair
mkdir -p $O
run() { local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  for g in 256 64 16; do
    CHM_REPAIR_GRID=$g run 64_g${g}_$rep --steps 30 --n-samples 64 || exit 1
  done
done
for g in 256 64; do CHM_REPAIR_GRID=$g run 512_g${g} --steps 10 || exit 1; done
cd /tmp && export TMPDIR=/tmp
for g in 256 64 16; do
  CHM_REPAIR_GRID=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/p$g -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --n-samples 64 --steps 5 --warmup 2 --no-cpu-baseline --no-api-legs > $GRAFT_REPO_ROOT/$O/p$g.log 2>&1 || exit 1
  grep repair $GRAFT_REPO_ROOT/$O/p$g/run_kernel_stats.csv | cut -d, -f1-4
done
