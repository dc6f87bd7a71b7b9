# SQ counters of the 2^25 Merkle leaf kernel (tools/bench_merkle.py 25): where its issue cycles go
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
rm -rf $R/gpurun_out/pmc_mk_sq
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mk_sq -o run -- python3 $R/tools/bench_merkle.py 25 > $R/gpurun_out/pmc_mk_sq.log 2>&1
f=$(ls $R/gpurun_out/pmc_mk_sq/*counter_collection.csv | head -1); python3 $R/tools/pmc_csv.py $f merkle
