set -e
mkdir -p gpurun_out/s2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu_sharded.py tests/test_gpu_configs.py > gpurun_out/s2/pytest.log 2>&1 || { tail -60 gpurun_out/s2/pytest.log; exit 1; }
tail -3 gpurun_out/s2/pytest.log
GDD_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/s2/bench2.log 2>&1 || { tail -40 gpurun_out/s2/bench2.log; exit 1; }
tail -1 gpurun_out/s2/bench2.log
timeout -k 10 400 python tools/bench_products.py > gpurun_out/s2/products.log 2>&1 || { tail -30 gpurun_out/s2/products.log; exit 1; }
tail -1 gpurun_out/s2/products.log
