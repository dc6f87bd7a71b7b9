set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tl -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > $R/gpurun_out/tl.log 2>&1
