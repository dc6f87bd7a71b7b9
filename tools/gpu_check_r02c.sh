# multi-GPU C ABI parity (sg_dist_*): world 1 over RCCL, 2/4/8 ranks on one GPU over a host transport
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 600 --timeout-method thread > gpurun_out/pt_dist.log 2>&1
