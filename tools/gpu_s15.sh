#!/bin/bash
# One-workgroup persistent k-means++ rounds: parity first (bounded), then timings and bench.
set -e
OUT=gpurun_out/s15
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_kpp.py > "$OUT/pytest_kpp.log" 2>&1 || { tail -60 "$OUT/pytest_kpp.log"; exit 1; }
tail -1 "$OUT/pytest_kpp.log"
timeout -k 10 600 $PYT tests/test_gpu_kmeans.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_agent.py > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python tools/micro_kpp.py > "$OUT/kpp.log" 2>&1 || { tail -30 "$OUT/kpp.log"; exit 1; }
cat "$OUT/kpp.log"
timeout -k 10 200 python tools/stamps.py > "$OUT/stamps.log" 2>&1 || { tail -30 "$OUT/stamps.log"; exit 1; }
grep kpp "$OUT/stamps.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
