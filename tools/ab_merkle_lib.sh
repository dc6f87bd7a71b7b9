# 2^25 Merkle tree build (tools/bench_merkle.py): ab/libstarkgpu_base.so vs the in-tree build, interleaved
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  echo "== base"; SG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libstarkgpu_base.so timeout -k 10 120 python tools/bench_merkle.py 25 2>&1 | tail -n 4
  echo "== new"; timeout -k 10 120 python tools/bench_merkle.py 25 2>&1 | tail -n 4
done
