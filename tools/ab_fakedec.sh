set -e
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  echo "== real"; timeout -k 10 120 python tools/bench_merkle.py 25 2>&1 | tail -n 4
  echo "== fake decimal"; SG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libstarkgpu_fakedec.so timeout -k 10 120 python tools/bench_merkle.py 25 2>&1 | tail -n 4
done
