# bf16x3 node GEMMs on 64-row tiles where the 128-row grid is short of the CUs (heads, conditioning): the
# microbenchmark (bit-identity + time), the GPU parity suite, then a same-box A/B against the previous library.
set -e
O=gpurun_out/b3rows
mkdir -p $O
for MKN in "2560 512 128" "5120 512 128" "10240 512 128" "128 640 1024" "1024 640 1024"; do
  set -- $MKN
  timeout -k 10 60 tools/gemm_bench $1 $2 b3rows $3 >> $O/micro.txt 2>&1
done
cat $O/micro.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_torch_ops.py \
  > $O/tests.txt 2>&1 || { tail -n 30 $O/tests.txt; exit 1; }
tail -n 2 $O/tests.txt
bash tools/ab.sh b3_6420 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 20 --steps 30 | tee $O/ab6420.txt
bash tools/ab.sh b3_64 3 "CHM_LIB=abl/base/libchemeleon_hip.so" "CHM_X=0" -- --n-samples 64 --n-atoms 40 --steps 20 | tee $O/ab64.txt
