#!/bin/bash
# Ordered-fold id prefetch + pipelined column chain: parity, fold micro, Lloyd at products, bench.
set -e
OUT=gpurun_out/s13
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 500 $PYT tests/test_gpu_kmeans.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_sharded.py > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python tools/micro_fold.py > "$OUT/fold.log" 2>&1 || { tail -30 "$OUT/fold.log"; exit 1; }
cat "$OUT/fold.log"
timeout -k 10 200 python tools/micro_cmean.py > "$OUT/cmean.log" 2>&1 || { tail -30 "$OUT/cmean.log"; exit 1; }
tail -3 "$OUT/cmean.log"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lloyd" -o lloyd \
  -- python3 tools/prof_lloyd.py > "$OUT/lloyd.log" 2>&1 || { tail -30 "$OUT/lloyd.log"; exit 1; }
grep KMeans "$OUT/lloyd.log"
timeout -k 10 300 python tools/bench_products.py > "$OUT/products.log" 2>&1 || { tail -30 "$OUT/products.log"; exit 1; }
tail -1 "$OUT/products.log"
