#!/bin/bash
# rocprofv3 kernel-trace summary of the bench + phase breakdown (each GPU step time-limited).
set -e
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python tools/phase_times.py > gpurun_out/phases.log 2>&1 || { tail -20 gpurun_out/phases.log; exit 1; }
cat gpurun_out/phases.log | grep rep
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
