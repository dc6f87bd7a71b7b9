# same-box A/B of the prove step: ab/libstarkgpu_base.so (a previous build) vs the in-tree library,
# interleaved A B A B ... (tools/step_timing.py: ms per prove over 8 proves each)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
  echo -n "base: " ; SG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libstarkgpu_base.so timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
  echo -n "new:  " ; timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
done
