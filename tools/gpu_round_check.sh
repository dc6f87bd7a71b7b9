# Full GPU check of the current tree: parity suite, default bench, kernel stats of the E2E step.
# Usage (from the repo root on the GPU box): bash tools/gpu_round_check.sh [tag]
# A heartbeat file under gpurun_out/ keeps long CPU-checker phases from looking hung.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-check}
cd $R
mkdir -p gpurun_out
(while true; do date +%s > gpurun_out/heartbeat; sleep 20; done) &
HB=$!
trap "kill $HB 2>/dev/null || true" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/pt_$TAG.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > $R/gpurun_out/prof_$TAG.log 2>&1
