# quick iteration: full GPU parity suite, NTT sizes, E2E bench (no side measurements)
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_pt.log 2>&1
rm -f gpurun_out/q_ntt.log
for n in 22 25; do timeout -k 10 120 python tools/bench_ntt.py $n >> gpurun_out/q_ntt.log 2>&1; done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-side > gpurun_out/q_e2e.log 2>&1
