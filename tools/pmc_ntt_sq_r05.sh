# Fresh SQ passes of the shipped NTT passes (round-5 verdict item 1): C2 (tools/bench_ntt.py 22)
# and inside the headline prove (tools/prove_only.py 3), two counter groups each, one run per group.
#   bash tools/pmc_ntt_sq_r05.sh            -> gpurun_out/pmc5_{c2,prove}_{1,2}/ + summaries
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
S1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
S2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAVES"
run() {  # name group-index counters... -- command...
  local name=$1; shift
  local d=$R/gpurun_out/pmc5_$name
  rm -rf $d
  timeout -s KILL ${PMC_LIMIT:-120} rocprofv3 --kernel-trace --pmc "$@" > $d.log 2>&1
}
for g in 1 2; do
  eval C=\$S$g
  run c2_$g $C --output-format csv -d $R/gpurun_out/pmc5_c2_$g -o run -- python3 $R/tools/bench_ntt.py 22
  run prove_$g $C --output-format csv -d $R/gpurun_out/pmc5_prove_$g -o run -- python3 $R/tools/prove_only.py 3
done
for n in c2 prove; do
  for g in 1 2; do
    f=$(ls $R/gpurun_out/pmc5_${n}_$g/*counter_collection.csv | head -1)
    echo "== $n pass $g"
    python3 $R/tools/pmc_csv.py $f k_ntt_
  done
done > $R/gpurun_out/pmc5_ntt_sq_summary.txt
