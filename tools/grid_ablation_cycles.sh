# The pair grid's CHM_EDGE_DBG ablations (tools/grid_ablation.sh) in cycles as well as time: an ablation changes the
# data the kernels see (e.g. S never written), and the chip's clock follows the data (MI355X_MICROARCH.md, DVFS), so
# a wall-time difference alone can be a clock artifact. One rocprofv3 pass per variant, GRBM_GUI_ACTIVE (summed over
# the 8 XCDs) per dispatch + the kernel trace; repo root, GPU box: bash tools/grid_ablation_cycles.sh <tag> [bench args]
# (from r6 the epilogue bits 4 and 524288 act only in an A/B build: CHM_BUILD_DEFS=-DCHM_PAIR_ABL=1, run with CHM_LIB)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
for d in ${GRID_DBG:-0 4 16 524288 4194304}; do
  CHM_EDGE_DBG=$d timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $O/d$d -o run --output-format csv \
    -- python3 $R/bench.py --traffic-probe "$@" > $O/d$d.log 2>&1 || { echo "dbg $d failed"; tail -5 $O/d$d.log; exit 1; }
  python3 $R/tools/cycles_summary.py $O/d$d "dbg $d"
done
