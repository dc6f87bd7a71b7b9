# SQ passes of the shipped Merkle kernels (k_merkle_leaf_pairs, k_merkle_levels<false,256>) on a
# 2^25-leaf tree (tools/bench_merkle.py 25): where their wave cycles go.  Each pass is its own
# rocprofv3 run (<= 8 SQ counters + GRBM).  Usage: bash tools/pmc_sq_merkle_v2.sh [tag]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-v2}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
pass() {
  name=$1; shift
  rm -rf $R/gpurun_out/pmc_sq_${TAG}_$name
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_sq_${TAG}_$name -o run \
    -- python3 $R/tools/bench_merkle.py 25 > $R/gpurun_out/pmc_sq_${TAG}_$name.log 2>&1
  f=$(ls $R/gpurun_out/pmc_sq_${TAG}_$name/*counter_collection.csv | head -1)
  python3 $R/tools/pmc_csv.py $f merkle > $R/gpurun_out/pmc_sq_${TAG}_$name.txt
}
pass wait SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
pass mix SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
