#!/bin/bash
# Hop changes: parity tests, bench line, PMC passes of k_hop at the arxiv (bench) and products
# (micro_reorder) shapes. Each GPU step time-limited; the first failure ends the script.
set -e
TAG=${1:-hop}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_graph.py tests/test_gpu_golden.py tests/test_gpu_gcn.py tests/test_gpu_configs.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_hop --output-format csv -d "$OUT/arxiv/pmc_fetch" -o bench -- $B > "$OUT/a1.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_hop --output-format csv -d "$OUT/arxiv/pmc_write" -o bench -- $B > "$OUT/a2.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_hop --output-format csv -d "$OUT/arxiv/pmc_hit" -o bench -- $B > "$OUT/a3.log" 2>&1
timeout -k 10 300 python -u tools/micro_reorder.py products orig > "$OUT/products_time.log" 2>&1
cat "$OUT/products_time.log" | grep us/hop
P="python3 tools/micro_reorder.py products orig"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_hop --output-format csv -d "$OUT/products/pmc_fetch" -o bench -- $P > "$OUT/p1.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_hop --output-format csv -d "$OUT/products/pmc_write" -o bench -- $P > "$OUT/p2.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_hop --output-format csv -d "$OUT/products/pmc_hit" -o bench -- $P > "$OUT/p3.log" 2>&1
find "$OUT" -name "*counter_collection.csv" | sort
