# SQ counters of the NTT passes (2^22 and 2^25 fwd+inv): where the issue slots go
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pmc_ntt_sq1 $R/gpurun_out/pmc_ntt_sq2
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/pmc_ntt_sq1 -o run -- python3 $R/tools/bench_ntt.py 25 > $R/gpurun_out/pmc_ntt_sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_ntt_sq2 -o run -- python3 $R/tools/bench_ntt.py 25 > $R/gpurun_out/pmc_ntt_sq2.log 2>&1
