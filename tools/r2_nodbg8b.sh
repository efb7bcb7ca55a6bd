# Second A/B at 64x40 and 512x40: previous build / no select in both epilogues / layer-1 epilogue only.
O=gpurun_out/nodbg8b
mkdir -p $O
run() { local tag=$1 lib=$2; shift 2
  CHM_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-api-legs "$@" > $O/$tag.log 2>&1 || return 1
  echo "$tag $(python tools/bench_summary.py $O/$tag.log)"; }
for rep in 1 2 3; do
  run 64_old_$rep abl/lib_new.so --steps 30 --n-samples 64 || exit 1
  run 64_both_$rep abl/lib_nodbg8.so --steps 30 --n-samples 64 || exit 1
  run 64_l1_$rep abl/lib_l1only.so --steps 30 --n-samples 64 || exit 1
done
for rep in 1 2; do
  run 512_old_$rep abl/lib_new.so --steps 10 || exit 1
  run 512_both_$rep abl/lib_nodbg8.so --steps 10 || exit 1
  run 512_l1_$rep abl/lib_l1only.so --steps 10 || exit 1
done
