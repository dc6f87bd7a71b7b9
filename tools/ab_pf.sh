# A/B: persistent NTT pass with next-tile prefetch during the last step (SG_NTT_PF) vs one tile per block
set -e
cd $GRAFT_REPO_ROOT
L=$PWD/zk-stark-tutor_amd/starkgpu
for cfg in "libstarkgpu.so 0" "libstarkgpu.so 1" "libstarkgpu_pf2.so 1"; do
  set -- $cfg
  echo "== $1 SG_NTT_PF=$2"
  SG_LIB_PATH=$L/$1 SG_NTT_PF=$2 timeout -k 10 100 python tools/bench_ntt.py 22
  SG_LIB_PATH=$L/$1 SG_NTT_PF=$2 timeout -k 10 100 python tools/bench_ntt.py 25
done
