# Same-box A/B of launch options: bench.py under each environment setting in turn, R rounds alternating
# (A B C A B C ...), so box drift hits every arm alike. Repo root, GPU box.
#   bash tools/ab.sh <tag> <rounds> "<env A>" "<env B>" ... -- <bench args>
# e.g. bash tools/ab.sh pool 2 "CHM_EDGE_POOL=15" "CHM_EDGE_POOL=0" -- --n-samples 64 --steps 20
# Prints one summary line per run (tools/bench_summary.py) and the per-arm median ms/step.
TAG=$1; R=$2; shift 2
ARMS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ARMS+=("$1"); shift; done
[ "$1" = "--" ] && shift
O=gpurun_out/ab_$TAG
mkdir -p $O
for r in $(seq 1 $R); do
  for i in "${!ARMS[@]}"; do
    f=$O/arm${i}_r${r}.json
    env ${ARMS[$i]} timeout -k 10 300 python bench.py --no-api-legs --no-cpu-baseline --no-traffic --warmup 3 "$@" \
      > $f 2> $f.err || { tail -n 20 $f.err; exit 1; }
    echo "[${ARMS[$i]}] $(python tools/bench_summary.py $f | head -1)"
  done
done
python - "$O" "${#ARMS[@]}" "${ARMS[@]}" <<'PY'
import glob, json, statistics, sys
o, n = sys.argv[1], int(sys.argv[2])
for i, arm in enumerate(sys.argv[3:3 + n]):
    ms = [json.loads([l for l in open(f) if l.startswith("{")][-1])["ms_per_step"] for f in sorted(glob.glob(f"{o}/arm{i}_r*.json"))]
    print(f"arm {i} [{arm}]: median {statistics.median(ms):.3f} ms/step over {len(ms)} runs: {' '.join(f'{m:.3f}' for m in ms)}")
PY
