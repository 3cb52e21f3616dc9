#!/bin/bash
# Re-entry check: a parity subset on the rebuilt library, the Lloyd kernel split at the products
# k-means shape (rocprofv3 stats), and the products-shape hot path after the assignment changes.
set -e
OUT=gpurun_out/s8
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_kpp.py tests/test_gpu_kmeans.py > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lloyd" -o lloyd \
  -- python3 tools/prof_lloyd.py > "$OUT/lloyd.log" 2>&1 || { tail -30 "$OUT/lloyd.log"; exit 1; }
grep KMeans "$OUT/lloyd.log"
timeout -k 10 300 python tools/bench_products.py > "$OUT/products.log" 2>&1 || { tail -30 "$OUT/products.log"; exit 1; }
tail -1 "$OUT/products.log"
find "$OUT" -name "*stats.csv" | sort
