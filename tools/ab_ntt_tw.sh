# A/B of the NTT twiddle plan: stage-major table vs computed high-stage twiddles, and a
# "free twiddles" timing bound (SG_NTT_TWMASK: wrong results, timing only)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_parity.log 2>&1
for lg in 22 25; do
  for cut in 30 22 20 18 16 12; do
    echo "== logn $lg TWCUT $cut" >> gpurun_out/ab_ntt.log
    SG_NTT_TWCUT=$cut timeout -k 10 120 python tools/bench_ntt.py $lg >> gpurun_out/ab_ntt.log 2>&1
  done
  echo "== logn $lg TWCUT 30 TWMASK 0xFF (free twiddles)" >> gpurun_out/ab_ntt.log
  SG_NO_CHECK=1 SG_NTT_TWCUT=30 SG_NTT_TWMASK=0xFF timeout -k 10 120 python tools/bench_ntt.py $lg >> gpurun_out/ab_ntt.log 2>&1
done
