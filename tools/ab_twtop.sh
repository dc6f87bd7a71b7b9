# prove (tools/step_timing.py) with the top SG_NTT_TWTOP stages' twiddles computed (default 3) vs
# read from the stage-major table, interleaved on one box
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for T in 3 0 1 2; do
    echo -n "TWTOP=$T: "; SG_NTT_TWTOP=$T timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
  done
done
