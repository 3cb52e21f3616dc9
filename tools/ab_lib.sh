#!/bin/bash
# Same-box A/B of two library builds on the bench line: tools/ab_lib.sh <tag> <libA> <libB> [rounds]
set -o pipefail
TAG=$1; A=$2; B=$3; R=${4:-3}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    echo "lib $L"
    GDD_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 > "$OUT/run.log" 2>&1 || { tail -20 "$OUT/run.log"; exit 1; }
    python3 -c "
import json,sys
d=[json.loads(l) for l in open('$OUT/run.log') if l.startswith('{')][-1]
print('  ms/step %.3f  kmeans %.3f  propagate %.3f' % (d['ms_per_step'], d['phases_ms']['kmeans'], d['phases_ms']['propagate']))"
  done
done
