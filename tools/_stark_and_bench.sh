set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_algebra.py tests/test_gpu_stark.py -q -m gpu -x > gpurun_out/stk.log 2>&1
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_e2e.log 2>&1
