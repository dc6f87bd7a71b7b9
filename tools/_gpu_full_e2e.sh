set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pt.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e2e -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > $R/gpurun_out/prof_e2e.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_e2e -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > $R/gpurun_out/pmc_fetch_e2e.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_e2e -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side > $R/gpurun_out/pmc_write_e2e.log 2>&1
