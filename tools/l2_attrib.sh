# Where k_edge16_layer_dyn's read excess comes from, run from the repo root on the
# GPU box: bash tools/l2_attrib.sh <tag> [bench args]
#  1. timing: the bench with the A operand of layer-1 / layer-2 / both tiles redirected to the first 16
#     row tiles (CHM_EDGE_DBG 32768 / 65536 / 98304: L2-resident, wrong results), against the product;
#  2. PMC over the 2-step eager probe: L2 hits / misses and the memory-side read requests by size and by
#     target (DRAM vs the Infinity Cache), for the product and for the two redirections.
# Then: python tools/l2_summary.py gpurun_out/<tag>
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for d in 0 32768 65536 98304; do
  CHM_EDGE_DBG=$d timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api-legs --no-traffic "$@" \
    > $O/bench_d$d.json 2> $O/bench_d$d.err || { tail -n 20 $O/bench_d$d.err; exit 1; }
  python tools/bench_summary.py $O/bench_d$d.json
done
cd /tmp
i=0
for spec in "0|TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" \
            "0|TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" \
            "0|FETCH_SIZE" \
            "32768|TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" \
            "65536|TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum"; do
  i=$((i+1))
  d=${spec%%|*}
  set=${spec#*|}
  CHM_EDGE_DBG=$d timeout -s KILL 150 rocprofv3 --pmc $set -d $O/pmc$i -o pmc$i --output-format csv -- \
    python3 $R/bench.py --traffic-probe "$@" > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -n 5 $O/pmc$i.log; exit 1; }
  echo "$d|$set" > $O/pmc$i/spec.txt
done
echo done
