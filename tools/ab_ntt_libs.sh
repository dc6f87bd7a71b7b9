# same-box A/B of NTT passes (tools/bench_ntt.py 22/25) and the prove step for several library builds
set -e
cd $GRAFT_REPO_ROOT
for lib in ${AB_LIBS:-ab/libstarkgpu_base.so zk-stark-tutor_amd/starkgpu/libstarkgpu.so}; do
  echo "== $lib"
  SG_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 100 python tools/bench_ntt.py 22
  SG_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 100 python tools/bench_ntt.py 25
  echo -n "prove: "; SG_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 150 python tools/step_timing.py 8 2>/dev/null | tail -n 1
done
