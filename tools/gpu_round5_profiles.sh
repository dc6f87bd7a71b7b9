# Round-5 evidence of the shipped build (the driver's gpurun commands of this round, kept for reuse):
# rocprofv3 kernel stats of the bench line, the three PMC passes (FETCH_SIZE, WRITE_SIZE,
# SQ_INSTS_VALU + GRBM_GUI_ACTIVE) reduced to profiles/r05_pmc_{traffic,valu}_e2e.json, and the
# device-memory fit checked at trace 2^22 / 2^23 (tools/mem_highwater.py).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
(while true; do date +%s > gpurun_out/heartbeat; sleep 20; done) &
HB=$!
trap "kill $HB 2>/dev/null || true" EXIT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_bench5
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench5 -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_bench5.json 2> $R/gpurun_out/prof_bench5.err
rm -f $R/gpurun_out/prof_bench5/run_kernel_trace.csv
cd $R
GRAFT_REPO_ROOT=$R bash tools/pmc_passes.sh
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_e2e/run_counter_collection.csv gpurun_out/pmc_write_e2e/run_counter_collection.csv gpurun_out/r5_pmc_traffic_e2e.json
python3 tools/pmc_valu.py gpurun_out/pmc_valu_e2e/run_counter_collection.csv profiles/r05_valu_mix.json gpurun_out/r5_pmc_valu_e2e.json
timeout -k 10 400 python3 tools/mem_highwater.py 22 23 > gpurun_out/r5_mem_highwater_22_23.log 2>&1
