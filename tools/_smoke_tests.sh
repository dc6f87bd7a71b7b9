set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pt.log 2>&1
