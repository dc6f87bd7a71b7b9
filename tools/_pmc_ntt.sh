set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc1 -o run -- python3 $R/tools/bench_ntt.py 22 > $R/gpurun_out/pmc1.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/pmc2 -o run -- python3 $R/tools/bench_ntt.py 22 > $R/gpurun_out/pmc2.log 2>&1
