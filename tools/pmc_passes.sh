# PMC passes of the E2E step: FETCH_SIZE / WRITE_SIZE / VALU, one counter group per run; then
# reduce locally: tools/pmc_traffic.py (HBM bytes per lane) and tools/pmc_valu.py (VALU per wave)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side"
rm -rf $R/gpurun_out/pmc_fetch_e2e $R/gpurun_out/pmc_write_e2e $R/gpurun_out/pmc_valu_e2e
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_e2e -o run -- python3 $B > $R/gpurun_out/pmc_fetch_e2e.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_e2e -o run -- python3 $B > $R/gpurun_out/pmc_write_e2e.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_valu_e2e -o run -- python3 $B > $R/gpurun_out/pmc_valu_e2e.log 2>&1
