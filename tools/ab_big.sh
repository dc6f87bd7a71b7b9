# NTT tile-size experiment (SG_NTT_BIG = 0 / 12 / 13; run against the experiment build that read SG_NTT_BIG): C2-style timings at 2^20, 2^22, 2^25, interleaved,
# then the NTT/LDE parity tests under each big-tile plan
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for B in 0 12 13; do
    for L in 20 22 25; do
      SG_NTT_BIG=$B timeout -k 10 120 python tools/c2_time.py $L 2>&1 | tail -n 1
    done
  done
done
for B in 12 13; do
  SG_NTT_BIG=$B timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -n 2
done
