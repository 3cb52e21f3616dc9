set -e
mkdir -p gpurun_out/ro3
export GDD_HOP_SCHED=1
timeout -k 10 200 python -u tools/micro_reorder.py arxiv orig degree > gpurun_out/ro3/arxiv_g16.log 2>&1
GDD_HOP_LANES=32 timeout -k 10 200 python -u tools/micro_reorder.py arxiv orig degree > gpurun_out/ro3/arxiv_g32.log 2>&1
GDD_HOP_LANES=32 timeout -k 10 400 python -u tools/micro_reorder.py products orig degree > gpurun_out/ro3/products_g32.log 2>&1
grep -H us/hop gpurun_out/ro3/*.log
