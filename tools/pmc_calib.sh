# FETCH_SIZE / WRITE_SIZE calibration passes over tools/pmc_calib (known byte counts per kernel).
# Usage (GPU box, repo root): bash tools/pmc_calib.sh
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $R/gpurun_out/pmc_calib_$c
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/gpurun_out/pmc_calib_$c -o run \
    -- $R/tools/pmc_calib > $R/gpurun_out/pmc_calib_$c.log 2>&1
  f=$(ls $R/gpurun_out/pmc_calib_$c/*counter_collection.csv | head -1)
  python3 $R/tools/pmc_csv.py $f k_ > $R/gpurun_out/pmc_calib_$c.txt
done
cat $R/gpurun_out/pmc_calib_FETCH_SIZE.txt $R/gpurun_out/pmc_calib_WRITE_SIZE.txt
