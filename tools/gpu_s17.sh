#!/bin/bash
set -e
OUT=gpurun_out/s17
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in 0 8 16 32 0; do
  if [ "$L" = "0" ]; then unset GDD_HOP_LANES; else export GDD_HOP_LANES=$L; fi
  echo "lanes=$L" >> "$OUT/prop.log"
  timeout -k 10 200 python tools/micro_prop.py >> "$OUT/prop.log" 2>&1 || { tail -30 "$OUT/prop.log"; exit 1; }
done
grep -v amdgpu.ids "$OUT/prop.log"
