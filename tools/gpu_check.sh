#!/bin/bash
# One GPU session: build check, parity tests, smoke, short bench. Each GPU step has its own limit.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
