# Epilogues without the per-element profiling select (dbg bit 3): bit-identity against the previous
# build (abl/lib_new.so) and alternating benches.
O=gpurun_out/nodbg8
mkdir -p $O
CHM_LIB=abl/lib_new.so timeout -k 10 200 python tools/node_da_check.py $O/old.pt > $O/check.log 2>&1 || { tail -5 $O/check.log; exit 1; }
CHM_LIB=abl/lib_nodbg8.so timeout -k 10 200 python tools/node_da_check.py $O/new.pt $O/old.pt >> $O/check.log 2>&1 || { tail -5 $O/check.log; exit 1; }
tail -1 $O/check.log
run() { local tag=$1 lib=$2; shift 2
  CHM_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2; do
  run 512_old_$rep abl/lib_new.so --steps 10 || exit 1
  run 512_new_$rep abl/lib_nodbg8.so --steps 10 || exit 1
  run 64_old_$rep abl/lib_new.so --steps 20 --n-samples 64 || exit 1
  run 64_new_$rep abl/lib_nodbg8.so --steps 20 --n-samples 64 || exit 1
done
