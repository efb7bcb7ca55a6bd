# rocprofv3 kernel-trace summary of a short bench run (run from the repo root on the GPU box).
# Optional args are passed to bench.py; PROF_DIR names the output directory under gpurun_out/.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${PROF_DIR:-prof}
mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $D/bench.log 2>&1
