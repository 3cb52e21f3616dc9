set -e
mkdir -p gpurun_out/ro2
for s in 0 1; do
  GDD_HOP_SCHED=$s timeout -k 10 200 python -u tools/micro_reorder.py arxiv orig degree > gpurun_out/ro2/arxiv_s$s.log 2>&1
done
GDD_HOP_SCHED=1 timeout -k 10 400 python -u tools/micro_reorder.py products orig degree > gpurun_out/ro2/products_s1.log 2>&1
GDD_HOP_LANES=32 timeout -k 10 400 python -u tools/micro_reorder.py products orig > gpurun_out/ro2/products_l32.log 2>&1
GDD_HOP_LANES=8 timeout -k 10 400 python -u tools/micro_reorder.py products orig > gpurun_out/ro2/products_l8.log 2>&1
grep -h us/hop gpurun_out/ro2/*.log
