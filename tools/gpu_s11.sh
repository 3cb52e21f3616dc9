#!/bin/bash
set -e
OUT=gpurun_out/s11
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu_kpp.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python tools/micro_kpp.py > "$OUT/kpp.log" 2>&1 || { tail -30 "$OUT/kpp.log"; exit 1; }
cat "$OUT/kpp.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
