# NTT A/B: parity of the transforms, then per-size timing with the register-direct pass on/off
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_algebra.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pt.log 2>&1
rm -f gpurun_out/ab_ntt.log
for rr in 1 0; do for n in 20 22 25; do echo "RR=$rr" >> gpurun_out/ab_ntt.log; SG_NTT_RR=$rr timeout -k 10 120 python tools/bench_ntt.py $n >> gpurun_out/ab_ntt.log 2>&1; done; done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-side > gpurun_out/ab_e2e.log 2>&1
