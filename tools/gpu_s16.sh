#!/bin/bash
set -e
OUT=gpurun_out/s16
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_kpp.py > "$OUT/pytest_kpp.log" 2>&1 || { tail -60 "$OUT/pytest_kpp.log"; exit 1; }
tail -1 "$OUT/pytest_kpp.log"
timeout -k 10 200 python tools/micro_kpp.py > "$OUT/kpp.log" 2>&1 || { tail -30 "$OUT/kpp.log"; exit 1; }
head -4 "$OUT/kpp.log"
timeout -k 10 200 python tools/stamps.py > "$OUT/stamps.log" 2>&1 || { tail -30 "$OUT/stamps.log"; exit 1; }
grep kpp "$OUT/stamps.log"
