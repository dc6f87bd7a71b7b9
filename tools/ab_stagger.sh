# A/B of the NTT first-round stagger (SG_NTT_STAGGER x s_sleep(32) on blocks with bit SG_NTT_STAGGER_BIT set)
set -e
cd $GRAFT_REPO_ROOT
for cfg in "0 8" "2 8" "4 8" "8 8" "4 0" "4 9"; do
  set -- $cfg
  echo "== SG_NTT_STAGGER=$1 SG_NTT_STAGGER_BIT=$2"
  SG_NTT_STAGGER=$1 SG_NTT_STAGGER_BIT=$2 SG_NO_CHECK=1 timeout -k 10 100 python tools/bench_ntt.py 22
  SG_NTT_STAGGER=$1 SG_NTT_STAGGER_BIT=$2 SG_NO_CHECK=1 timeout -k 10 100 python tools/bench_ntt.py 25
done
