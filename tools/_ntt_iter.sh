# NTT iteration: parity, per-size timing, E2E bench, SQ counters of the 2^25 transform
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_algebra.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_pt.log 2>&1
for n in 20 22 24 25; do timeout -k 10 120 python tools/bench_ntt.py $n >> gpurun_out/nt_bench.log 2>&1; done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-side > gpurun_out/nt_e2e.log 2>&1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmcA $R/gpurun_out/pmcB
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcA -o run -- python3 $R/tools/bench_ntt.py 25 > $R/gpurun_out/pmcA.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/pmcB -o run -- python3 $R/tools/bench_ntt.py 25 > $R/gpurun_out/pmcB.log 2>&1
