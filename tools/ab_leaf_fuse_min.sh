# same-box sweep: smallest leaf level whose launch also fuses node levels (SG_MERKLE_LEAF_FUSE_MIN
# = log2; below it the leaf launch hashes leaves only), interleaved
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for fm in 12 15 18; do
    echo -n "fuse_min=2^$fm: " ; SG_MERKLE_LEAF_FUSE_MIN=$fm timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
  done
done > gpurun_out/ab_leaf_fuse_min.log
