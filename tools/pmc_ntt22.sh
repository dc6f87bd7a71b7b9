# SQ counters of the 2^22 NTT passes (tools/bench_ntt.py 22): where a pass's wave cycles go
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_MISC" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_IFETCH TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  rm -rf $R/gpurun_out/pmc22_$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/pmc22_$i -o run -- python3 $R/tools/bench_ntt.py ${NTT_LOG:-22} > $R/gpurun_out/pmc22_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc22_$i.log; }
done
for i in 1 2 3; do f=$(ls $R/gpurun_out/pmc22_$i/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 $R/tools/pmc_csv.py $f ntt; done
