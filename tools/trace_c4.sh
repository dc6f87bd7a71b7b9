# kernel trace + phase marks of the C4 prove (Rescue-Prime trace 2^16): where a latency-bound prove spends time
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/c4prof
SG_PROVE_TIMING=1 timeout -k 10 200 python3 $R/tools/prove_only.py 3 16 > $R/gpurun_out/c4_phases.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c4prof -o run -- python3 $R/tools/prove_only.py 4 16 > $R/gpurun_out/c4prof.log 2>&1
