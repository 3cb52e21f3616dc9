#!/bin/bash
# Pipelined LDS chains (centring fold, k-means++ sgemv lanes): parity, micro timings, bench.
set -e
OUT=gpurun_out/s10
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 500 $PYT tests/test_gpu_kpp.py tests/test_gpu_kmeans.py tests/test_gpu_golden.py tests/test_gpu_configs.py > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python tools/micro_kpp.py > "$OUT/kpp.log" 2>&1 || { tail -30 "$OUT/kpp.log"; exit 1; }
cat "$OUT/kpp.log"
timeout -k 10 200 python tools/micro_center.py > "$OUT/center.log" 2>&1 || { tail -30 "$OUT/center.log"; exit 1; }
cat "$OUT/center.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-400
