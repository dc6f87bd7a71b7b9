# E2E diagnosis: GPU parity suite, bench, host phase marks, kernel trace of the prove
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/d_pt.log 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-side > gpurun_out/d_e2e.log 2>&1
SG_PROVE_TIMING=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/d_phase.log 2>&1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/d_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/d_prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > $R/gpurun_out/d_prof.log 2>&1
