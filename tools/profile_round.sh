# Round-end measurements (repo root, GPU box): rocprofv3 kernel statistics of short bench runs at 512x40
# and 64x40, PMC passes of the dominant kernel (MFMA busy cycles + clock, LDS bank conflicts; the HBM
# traffic passes run inside bench.py itself), the BASELINE configs on one GPU and the ragged C4 run.
# Usage: bash tools/profile_round.sh <tag>   (outputs in gpurun_out/<tag>/)
T=${1:-final}
R=$PWD
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-api-legs --no-traffic"
for ns in 512 64; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof$ns -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 $B --n-samples $ns > $O/prof$ns.log 2>&1) || { tail -n 20 $O/prof$ns.log; exit 1; }
  find $O/prof$ns -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_${ns}x40.csv \;
done
(cd /tmp && timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $O/p1 -o p1 \
  --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 $B --no-graph > $O/p1.log 2>&1) || { tail -n 20 $O/p1.log; exit 1; }
(cd /tmp && timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/p2 -o p2 --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 1 $B --no-graph > $O/p2.log 2>&1) || { tail -n 20 $O/p2.log; exit 1; }
python tools/pmc_summary.py $O/p1 $O/p2 | grep -E "edge16_layer|k_node_gemm|counter_collection" > $O/pmc_summary.txt
for cfg in "64x20:--n-samples 64 --n-atoms 20" "256x40:--n-samples 256" "64x40:--n-samples 64" "128x40:--n-samples 128"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 python bench.py $B $a > $O/bench_$n.json 2> $O/bench_$n.err || { tail -n 20 $O/bench_$n.err; exit 1; }
  echo "$n $(python tools/bench_summary.py $O/bench_$n.json | head -1)"
done
timeout -k 10 400 python bench.py $B --ragged --n-samples 2048 --steps 3 --warmup 1 > $O/bench_c4_2048.json 2> $O/bench_c4.err \
  || { tail -n 20 $O/bench_c4.err; exit 1; }
echo "c4_2048 $(python tools/bench_summary.py $O/bench_c4_2048.json | head -1)"
echo "=== done"
