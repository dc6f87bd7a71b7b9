# A/B of the persistent NTT pass: per-pass times at 2^22 / 2^25 for grid knobs, then the prove
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in -1 0 1; do
  echo "== SG_NTT_PERSIST=$k"
  SG_NTT_PERSIST=$k SG_NO_CHECK=0 timeout -k 10 100 python tools/bench_ntt.py 22
  SG_NTT_PERSIST=$k timeout -k 10 100 python tools/bench_ntt.py 25
done
for k in -1 0; do
  echo "== prove SG_NTT_PERSIST=$k"
  SG_NTT_PERSIST=$k timeout -k 10 200 python tools/prove_only.py 5
done
