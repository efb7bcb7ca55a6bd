# Rehearse bench.py's multi-rank path (rank sharding, conditioning broadcast, barrier, max-over-ranks
# timing, final all-gather) on ONE GPU: 2 ranks share it over gloo. Repo root, GPU box.
mkdir -p gpurun_out
CHM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus ${NP:-2} --steps 2 --warmup 1 --no-cpu-baseline \
  --n-samples 64 "$@" > gpurun_out/dist_rehearsal.log 2>&1 || { tail -n 30 gpurun_out/dist_rehearsal.log; exit 1; }
python tools/bench_summary.py gpurun_out/dist_rehearsal.log
