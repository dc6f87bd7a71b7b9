# parity of the NTT suite, then C2 / 2^25 NTT timing: previous library vs current (trivial first-step twiddles)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_parity.log 2>&1
rm -f gpurun_out/ab_first.log
for i in 1 2; do
  for v in prev cur; do
    if [ $v = prev ]; then L="SG_LIB_PATH=$GRAFT_REPO_ROOT/ab/libstarkgpu_prev.so"; else L="SG_X=1"; fi
    echo "== $v" >> gpurun_out/ab_first.log
    env $L timeout -k 10 120 python tools/bench_ntt.py 22 >> gpurun_out/ab_first.log 2>&1
  done
done
AB_VARIANTS="prev cur prev cur" bash tools/ab_bench.sh
