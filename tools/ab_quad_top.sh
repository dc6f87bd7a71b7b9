# same-box A/B: tree tops in 64-node quad blocks only (SG_MERKLE_QUAD_TOP=0) vs the last <= 256
# nodes of each tree in one 1024-lane block; then the GPU suite on the new default
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
  echo -n "top=0: " ; SG_MERKLE_QUAD_TOP=0 timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
  echo -n "top=1: " ; timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
done > gpurun_out/ab_quad_top.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
