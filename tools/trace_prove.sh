# kernel trace of the prove alone (tools/prove_only.py), for idle-gap / overlap analysis
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_prove
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_prove -o run -- python3 $R/tools/prove_only.py 4 > $R/gpurun_out/prof_prove.log 2>&1
SG_PROVE_TIMING=1 timeout -k 10 200 python3 $R/tools/prove_only.py 3 > $R/gpurun_out/prove_phases.log 2>&1
