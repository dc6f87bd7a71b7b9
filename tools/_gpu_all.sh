set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pt.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-side > $R/gpurun_out/prof.log 2>&1
