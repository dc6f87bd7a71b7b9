# latency-bound Merkle trees (2^9 .. 2^16 leaves, tools/bench_merkle.py): ab/libstarkgpu_base.so vs in-tree
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for L in 10 13 16; do
    echo -n "base 2^$L: "; SG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libstarkgpu_base.so timeout -k 10 120 python tools/bench_merkle.py $L 2>&1 | grep "ms/build"
    echo -n "new  2^$L: "; timeout -k 10 120 python tools/bench_merkle.py $L 2>&1 | grep "ms/build"
  done
done
