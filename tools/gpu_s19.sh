#!/bin/bash
set -e
OUT=gpurun_out/s19
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_golden.py tests/test_gpu_configs.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for L in 1 2 3 1; do
  echo "lookahead=$L" >> "$OUT/fit.log"
  GDD_MB_LOOKAHEAD=$L timeout -k 10 200 python tools/gap_fit.py >> "$OUT/fit.log" 2>&1 || { tail -30 "$OUT/fit.log"; exit 1; }
done
grep -v amdgpu.ids "$OUT/fit.log"
for L in 1 2; do
  GDD_MB_LOOKAHEAD=$L timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_$L.log" 2>&1 || { tail -30 "$OUT/bench_$L.log"; exit 1; }
  echo "bench lookahead=$L: $(tail -1 $OUT/bench_$L.log | cut -c150-260)"
done
