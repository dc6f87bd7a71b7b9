# NTT tile-size sweep (SG_NTT_BIG = 0 / 12 / 13; experiment build -- the library now plans by size, SG_NTT_TILES=0 disables) at 2^16 .. 2^21, interleaved twice
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for L in 16 17 18 19 20 21; do
    for B in 0 12 13; do
      SG_NTT_BIG=$B timeout -k 10 120 python tools/c2_time.py $L 2>&1 | tail -n 1
    done
  done
done
