# 2^25 Merkle tree build under the leaf-kernel plan knobs (block size, fused levels), two rounds
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for cfg in "512 4 4" "512 1 4" "512 2 4" "512 3 4" "256 4 4" "1024 4 4" "1024 5 4" "512 4 6"; do
    set -- $cfg
    echo -n "BS=$1 FUSE=$2 NODE_FUSE=$3: "
    SG_MERKLE_LEAF_BS=$1 SG_MERKLE_LEAF_FUSE=$2 SG_MERKLE_NODE_FUSE=$3 timeout -k 10 120 python tools/bench_merkle.py 25 2>&1 | grep "ms/build"
  done
done
