# round-2 check: parity suite, Merkle/NTT microbenches, LDS bank-conflict PMC pass, full bench
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
timeout -k 10 120 python tools/bench_merkle.py 25 1 > gpurun_out/bm25.log 2>&1
timeout -k 10 120 python tools/bench_ntt.py 22 > gpurun_out/bn22.log 2>&1
timeout -k 10 120 python tools/bench_ntt.py 25 > gpurun_out/bn25.log 2>&1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_lds
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_lds -o run -- python3 $R/tools/bench_merkle.py 25 1 > $R/gpurun_out/pmc_lds.log 2>&1
cd $R
timeout -k 10 500 python bench.py > gpurun_out/bench.log 2>&1
