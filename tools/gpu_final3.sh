#!/bin/bash
# Round-end session (r02, third part): whole -m gpu suite, smoke, bench line with the CPU baseline,
# rocprofv3 kernel stats of the bench, phase times, k-means++ micro, Reddit inductive shape.
set -e
TAG=${1:-final3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 1000 $PYT tests > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-200
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
timeout -k 10 300 python tools/phase_times.py > "$OUT/phases.log" 2>&1 || { tail -20 "$OUT/phases.log"; exit 1; }
timeout -k 10 200 python tools/micro_kpp.py > "$OUT/kpp.log" 2>&1 || { tail -30 "$OUT/kpp.log"; exit 1; }
timeout -k 10 300 python tools/bench_induct.py > "$OUT/reddit.log" 2>&1 || { tail -30 "$OUT/reddit.log"; exit 1; }
tail -1 "$OUT/reddit.log" | cut -c1-300
echo done
