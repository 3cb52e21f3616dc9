#!/bin/bash
# Lloyd single-init async return: parity suites touching KMeans, products shape, bench + kernel stats.
set -e
OUT=gpurun_out/s14
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 600 $PYT tests/test_gpu_kmeans.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_agent.py tests/test_gpu_recsys.py tests/test_gpu_edge.py > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python tools/bench_products.py > "$OUT/products.log" 2>&1 || { tail -30 "$OUT/products.log"; exit 1; }
tail -1 "$OUT/products.log"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log" | cut -c1-200
