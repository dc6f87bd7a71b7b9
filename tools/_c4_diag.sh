# C4 (trace 2^16) diagnosis: bench, host phase marks, kernel trace
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-side --log-trace 16 > gpurun_out/c4_e2e.log 2>&1
SG_PROVE_TIMING=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side --log-trace 16 > gpurun_out/c4_phase.log 2>&1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/c4_prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c4_prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side --log-trace 16 > $R/gpurun_out/c4_prof.log 2>&1
