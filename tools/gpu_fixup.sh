#!/bin/bash
# bounded split-row fix-up grid: propagation parity, hop micro, bench
set -e
OUT=gpurun_out/${1:-fixup}
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_graph.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_gcn.py tests/test_gpu_edge.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
grep -E "k_fixup|k_hop" "$OUT/trace/bench_kernel_stats.csv" | cut -c1-40,200-400 | cut -d, -f1-4 || true
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["phases_ms"].items()}, d["roofline"]["avg_launch_ms"])'
