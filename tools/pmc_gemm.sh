# PMC passes over the edge-GEMM microbenchmark (run from the repo root on the GPU box)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc
mkdir -p $O
timeout -k 10 120 $R/tools/gemm_bench 819200 768 edge > $O/plain.log 2>&1 &&
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/p1 -o p1 --output-format csv -- $R/tools/gemm_bench 819200 768 edge > $O/p1.log 2>&1 &&
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $O/p2 -o p2 --output-format csv -- $R/tools/gemm_bench 819200 768 edge > $O/p2.log 2>&1 &&
timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_TA_BUSY GRBM_GUI_ACTIVE -d $O/p3 -o p3 --output-format csv -- $R/tools/gemm_bench 819200 768 edge > $O/p3.log 2>&1 &&
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/p4 -o p4 --output-format csv -- $R/tools/gemm_bench 819200 768 edge > $O/p4.log 2>&1
