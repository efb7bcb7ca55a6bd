# MFMA busy cycles, effective clock and LDS bank conflicts of the one-grid edge-layer kernel
# (512x40, eager, one step), two separate rocprofv3 --pmc passes. Repo root on the GPU box.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_layer
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $O/p1 -o p1 --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-api-legs --no-graph > $O/p1.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/p2 -o p2 --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-api-legs --no-graph > $O/p2.log 2>&1 || exit 1
cd $R && python tools/pmc_summary.py $O/p1 $O/p2 | grep -E "edge16_layer|k_edge16<|counter_collection" | head -40 > $O/summary.txt; tail -12 $O/summary.txt
