# The epilogues' ablations in cycles (A/B build abl/epi: -DCHM_PAIR_ABL=1 -DCHM_L2_SEL=1; wrong results): the pair grid
# at 512x40 under CHM_EDGE_DBG 0, 16 (main loops only), 8 (no layer-2 SiLU), 32 (no segment sums), 40, 4 (no stores),
# 2097152 (no S exponent bytes). Repo root, GPU box.
O=$GRAFT_REPO_ROOT/gpurun_out/epic; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-0 16 8 32 40 4}; do
  CHM_LIB=$GRAFT_REPO_ROOT/abl/epi/libchemeleon_hip.so CHM_EDGE_DBG=$d timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE \
    --kernel-trace -d $O/d$d -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --traffic-probe --n-samples 512 \
    > $O/d$d.log 2>&1 || { tail -5 $O/d$d.log; exit 1; }
  python3 $GRAFT_REPO_ROOT/tools/cycles_summary.py $O/d$d "dbg $d" | head -1
done
