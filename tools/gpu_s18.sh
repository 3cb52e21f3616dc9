#!/bin/bash
set -e
OUT=gpurun_out/s18
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python tools/gap_fit.py > "$OUT/fit.log" 2>&1 || { tail -30 "$OUT/fit.log"; exit 1; }
cat "$OUT/fit.log"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o fit -- python3 tools/gap_fit.py > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
python3 tools/gap_report.py "$(find $OUT/trace -name '*kernel_trace.csv' | head -1)"
