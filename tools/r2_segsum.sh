# Segment sums with two columns per lane (one wave per node): bit-identity against the previous build
# (abl/lib_old.so) on a reverse step, the parity tests, then alternating benches old / new.
O=gpurun_out/segsum
mkdir -p $O
CHM_LIB=abl/lib_old.so timeout -k 10 200 python tools/node_da_check.py $O/old.pt > $O/check.log 2>&1 || { tail -5 $O/check.log; exit 1; }
CHM_LIB=abl/lib_new.so timeout -k 10 200 python tools/node_da_check.py $O/new.pt $O/old.pt >> $O/check.log 2>&1 || { tail -5 $O/check.log; exit 1; }
tail -1 $O/check.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "row_tiles or single_conditioning or at_size or decoder or trajectory or shard or segment" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
run() { local tag=$1 lib=$2; shift 2
  CHM_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  run 512_old_$rep abl/lib_old.so --steps 10 || exit 1
  run 512_new_$rep abl/lib_new.so --steps 10 || exit 1
  run 64_old_$rep abl/lib_old.so --steps 20 --n-samples 64 || exit 1
  run 64_new_$rep abl/lib_new.so --steps 20 --n-samples 64 || exit 1
done
