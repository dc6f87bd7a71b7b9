# arbitrary-domain algebra parity + the algebra/stark suites
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_algebra.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pt_alg.log 2>&1
