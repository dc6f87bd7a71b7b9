# kernel trace + phase marks of the C4 prove (Rescue-Prime trace 2^16): where a latency-bound prove
# spends time.  Phase marks need the A/B build (SG_PROVE_TIMING is an A/B knob since round 6); the
# trace runs the product library.  Then tools/critical_path.py lays out the chain kernel by kernel.
# usage (repo root on the GPU box): bash tools/trace_c4.sh [tag] [log_trace]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-c4}
L=${2:-16}
mkdir -p $R/gpurun_out
SG_LIB_PATH=$R/zk-stark-tutor_amd/starkgpu/libstarkgpu_ab.so SG_PROVE_TIMING=1 \
  timeout -k 10 200 python3 $R/tools/prove_only.py 3 $L > $R/gpurun_out/${TAG}_phases.log 2>&1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/${TAG}_prof
SG_PROVE_GAPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- \
  python3 $R/tools/prove_only.py 4 $L > $R/gpurun_out/${TAG}_prof.log 2>&1
python3 $R/tools/critical_path.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv 20 $R/gpurun_out/${TAG}_critical_path.json \
  > $R/gpurun_out/${TAG}_critical_path.txt 2>&1
