#!/bin/bash
set -e
OUT=gpurun_out/s12
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python tools/stamps.py > "$OUT/stamps.log" 2>&1 || { tail -30 "$OUT/stamps.log"; exit 1; }
cat "$OUT/stamps.log"
timeout -k 10 200 python tools/micro_fold.py > "$OUT/fold.log" 2>&1 || { tail -30 "$OUT/fold.log"; exit 1; }
cat "$OUT/fold.log"
