# Direct-A node GEMM (CHM_NODE_DA=1): bit-identity of a reverse step against the LDS-staged kernel,
# the decoder / step parity tests with it on, then alternating bench runs at 512x40 and 64x40.
O=gpurun_out/nodeda
mkdir -p $O
timeout -k 10 200 python tools/node_da_check.py $O/ref.pt > $O/check.log 2>&1 || { tail -5 $O/check.log; exit 1; }
CHM_NODE_DA=1 timeout -k 10 200 python tools/node_da_check.py $O/da.pt $O/ref.pt >> $O/check.log 2>&1 || { tail -5 $O/check.log; exit 1; }
tail -1 $O/check.log
CHM_NODE_DA=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "decoder_forward or teacher or at_size" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
run() { local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  run 512_base_$rep --steps 10 || exit 1
  CHM_NODE_DA=1 run 512_da_$rep --steps 10 || exit 1
  run 64_base_$rep --steps 20 --n-samples 64 || exit 1
  CHM_NODE_DA=1 run 64_da_$rep --steps 20 --n-samples 64 || exit 1
done
