#!/bin/bash
# One GPU session: the changed parity tests first (fail fast), then the whole -m gpu suite, smoke, a
# bench line (with the CPU baseline) and a rocprofv3 kernel-trace summary of a short bench.
# Each GPU step has its own time limit; the first failure ends the script.
# usage: tools/gpu_session.sh <tag> [first test files...]
set -e
TAG=${1:-s}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
if [ $# -gt 0 ]; then
  timeout -k 10 600 $PYT "$@" > "$OUT/pytest_first.log" 2>&1 || { tail -60 "$OUT/pytest_first.log"; exit 1; }
  tail -3 "$OUT/pytest_first.log"
fi
timeout -k 10 1000 $PYT tests > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py ${BENCH_ARGS} > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
find "$OUT" -name "*stats.csv" | sort
