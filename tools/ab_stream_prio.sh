# prove (tools/step_timing.py) with SG_STREAM_PRIO = 0 (default), 1 (side stream high), -1 (main high); needs the experiment build that read SG_STREAM_PRIO (profiles/r02_ab_stream_priority.log)
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for P in 0 1 -1; do
    echo -n "PRIO=$P: "; SG_STREAM_PRIO=$P timeout -k 10 150 python tools/step_timing.py ${AB_STEPS:-8} ${AB_LOG:-20} 2>/dev/null | tail -n 1
  done
done
