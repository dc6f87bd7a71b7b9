set -e
R=$GRAFT_REPO_ROOT
cd $R
SG_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench2.log 2>&1
