set -e
cd $GRAFT_REPO_ROOT
for v in "" _xp3; do
  echo "== lib$v"
  SG_LIB_PATH=$PWD/zk-stark-tutor_amd/starkgpu/libstarkgpu$v.so SG_NO_CHECK=1 timeout -k 10 100 python tools/bench_ntt.py 22
done
