# C2-style fwd+inv timings (tools/c2_time.py) at 2^20 / 2^22 / 2^25: ab/libstarkgpu_base.so vs the
# in-tree build, interleaved
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for L in 20 22 25; do
    echo -n "base: "; SG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libstarkgpu_base.so timeout -k 10 120 python tools/c2_time.py $L 2>&1 | tail -n 1
    echo -n "new:  "; timeout -k 10 120 python tools/c2_time.py $L 2>&1 | tail -n 1
  done
done
