# one iteration: GPU parity of the algebra + Stark paths, E2E bench, kernel trace of the E2E step
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_algebra.py tests/test_gpu_stark.py -q -m gpu -x > gpurun_out/stk.log 2>&1
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > gpurun_out/bench_e2e.log 2>&1
rm -rf gpurun_out/prof_it
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_it -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side > $R/gpurun_out/prof_it.log 2>&1
