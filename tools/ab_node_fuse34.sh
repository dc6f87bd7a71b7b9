# same-box A/B: 3 vs 4 node levels per one-lane-per-node launch (SG_MERKLE_NODE_FUSE), 4 pairs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for nf in 4 3; do
    echo -n "node_fuse=$nf: " ; SG_MERKLE_NODE_FUSE=$nf timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
  done
done > gpurun_out/ab_node_fuse34.log
