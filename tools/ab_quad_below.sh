# same-box sweep of the level size below which tree levels switch to quad-per-node blocks
# (SG_MERKLE_QUAD_BELOW = log2), interleaved; then the driver's smoke()
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for qb in 14 16 17 18; do
    echo -n "below=2^$qb: " ; SG_MERKLE_QUAD_BELOW=$qb timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
  done
done > gpurun_out/ab_quad_below.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
