# One GPU-box session of checks, run from the repo root: bash tools/gpu_round.sh <tag> <steps...>
# steps: tests=<pytest -k expr> | gputests (the whole -m gpu suite) | smoke | bench[:args] | dist2 | prof[:args]
# Every step runs under its own time limit; the first failure ends the session (no GPU step after a
# fault, abort or timeout). Outputs go to gpurun_out/<tag>/.
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%[:=]*}
  arg=${step#*[:=]}
  [ "$arg" = "$step" ] && arg=""
  echo "=== $step $(date +%T)"
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread -k "$arg" \
        > $O/tests_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40).txt 2>&1 || { tail -n 40 $O/tests_*.txt; exit 1; } ;;
    gputests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > $O/gputests.txt 2>&1 || { tail -n 40 $O/gputests.txt; exit 1; }
      tail -n 3 $O/gputests.txt ;;
    bench)
      f=$O/bench_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60).json
      timeout -k 10 600 python -u bench.py $arg > $f 2> $f.err || { tail -n 30 $f.err; exit 1; }
      python tools/bench_summary.py $f ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -n 20 $O/smoke.txt; exit 1; }
      tail -n 1 $O/smoke.txt ;;
    dist2)
      f=$O/dist2.json
      CHM_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --n-samples 64 --steps 2 --warmup 1 \
        --no-cpu-baseline $arg > $f 2> $f.err || { tail -n 30 $f.err; exit 1; }
      python tools/bench_summary.py $f ;;
    prof)
      D=$PWD/$O/prof_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
      mkdir -p $D
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- \
        python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api-legs --no-traffic $arg \
        > $D/bench.log 2>&1) || { tail -n 30 $D/bench.log; exit 1; }
      find $D -name '*kernel_stats.csv' -exec head -n 12 {} \; ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== done $(date +%T)"
