set -e
for cfg in "256 3 3" "256 3 4" "512 4 3" "512 4 4" "512 5 3"; do
  set -- $cfg
  SG_MERKLE_LEAF_BS=$1 SG_MERKLE_LEAF_FUSE=$2 SG_MERKLE_NODE_FUSE=$3 timeout -k 10 100 python tools/bench_merkle.py 23 3 >> gpurun_out/mk.txt 2>&1
  echo "node fuse $3" >> gpurun_out/mk.txt
done
