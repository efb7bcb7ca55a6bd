# Round-6 validation of the committed tree, one GPU box: the whole -m gpu suite, smoke, the default bench line,
# rocprofv3 kernel stats at 512x40 / 64x40 / 64x20. Repo root, GPU box: FINAL_TAG=<tag> bash tools/final_r6.sh
set -e
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/${FINAL_TAG:-final6}
mkdir -p $O
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { tail -n 40 $O/gputests.txt; exit 1; }
  tail -n 2 $O/gputests.txt
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
tail -n 1 $O/smoke.txt
timeout -k 10 420 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python tools/bench_summary.py $O/bench_default.json | head -3
cd /tmp && export TMPDIR=/tmp
for cfg in "512 40" "64 40" "64 20"; do
  set -- $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p$1x$2 -o run --output-format csv -- python3 $R/bench.py --n-samples $1 --n-atoms $2 --steps 5 --warmup 2 --no-cpu-baseline --no-api-legs --no-traffic > $O/bench_$1x$2.json 2> $O/bench_$1x$2.err
  python $R/tools/bench_summary.py $O/bench_$1x$2.json | head -1
done
