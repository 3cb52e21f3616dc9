#!/bin/bash
# One measurement round on the GPU box: phase breakdown, bench line, rocprofv3 kernel-trace stats of
# the bench, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE) restricted to the SpMM hop kernel.
# Every GPU step has its own time limit; the first failure ends the script.
# usage: tools/gpu_round.sh <tag>   (outputs under gpurun_out/<tag>/)
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/phase_times.py > "$OUT/phases.log" 2>&1 || { tail -20 "$OUT/phases.log"; exit 1; }
grep rep "$OUT/phases.log"
timeout -k 10 420 python bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_hop" --output-format csv -d "$OUT/pmc_fetch" -o bench \
  -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 || { tail -20 "$OUT/pmc_fetch.log"; exit 1; }
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_hop" --output-format csv -d "$OUT/pmc_write" -o bench \
  -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1 || { tail -20 "$OUT/pmc_write.log"; exit 1; }
find "$OUT" -name "*.csv" | sort
