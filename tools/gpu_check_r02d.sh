# C5 through the C ABI at 2^27 (world 2 and 8 on one GPU), then a world-2 gloo rehearsal of the
# bench's sharded side measurements and the default N=1 bench
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v -k "c5_native" --timeout 800 --timeout-method thread > gpurun_out/pt_c5native.log 2>&1
SG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_gloo2.log 2>&1
timeout -k 10 500 python bench.py --no-cpu-baseline > gpurun_out/bench_n1.log 2>&1
