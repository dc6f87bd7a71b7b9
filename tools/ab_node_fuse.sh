# same-box sweep of node levels fused per one-lane-per-node launch (SG_MERKLE_NODE_FUSE), with the
# one-block tree tops, interleaved
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for nf in 3 4 5; do
    echo -n "node_fuse=$nf: " ; SG_MERKLE_NODE_FUSE=$nf timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
  done
done > gpurun_out/ab_node_fuse.log
