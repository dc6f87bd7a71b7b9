set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_valu_e2e -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > $R/gpurun_out/pmc_valu_e2e.log 2>&1
