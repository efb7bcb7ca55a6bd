# Per-kernel SQ / LDS counters of the sampler's kernels over a 2-step eager probe (bench.py
# --traffic-probe), one rocprofv3 --pmc pass per counter set (gfx950 slot limits: <= 8 SQ, 2 GRBM).
# Run from the repo root on the GPU box: bash tools/pmc_kernels.sh <tag> [bench args]; then
# python tools/pmc_summary.py gpurun_out/<tag>
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/pass$i -o pass$i --output-format csv -- python3 $R/bench.py --traffic-probe "$@" > $O/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pass$i.log; }
done
echo done
