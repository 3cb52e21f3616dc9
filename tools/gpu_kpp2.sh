#!/bin/bash
# two-rounds-per-launch k-means++: parity tests, round A/B, bench line
set -e
OUT=gpurun_out/${1:-kpp2}
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_kpp.py tests/test_gpu_golden.py tests/test_gpu_kmeans.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python tools/micro_kpp.py > "$OUT/kpp.log" 2>&1 || { tail -30 "$OUT/kpp.log"; exit 1; }
grep -v amdgpu.ids "$OUT/kpp.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
