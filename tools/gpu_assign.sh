#!/bin/bash
# assignment kernels: timing, parity tests, MFMA PMC pass + kernel trace of tools/bench_assign.py
set -e
OUT=gpurun_out/${1:-assign}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 150 python tools/bench_assign.py > "$OUT/bench_assign.log" 2>&1 || { tail -20 "$OUT/bench_assign.log"; exit 1; }
tail -1 "$OUT/bench_assign.log"
timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu_kmeans.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_edge.py tests/test_gpu_sharded.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_assign" --output-format csv -d "$OUT/pmc_mfma" -o assign -- python3 tools/bench_assign.py > "$OUT/pmc_mfma.log" 2>&1 || { tail -20 "$OUT/pmc_mfma.log"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/assign_trace" -o assign -- python3 tools/bench_assign.py > "$OUT/assign_trace.log" 2>&1 || { tail -20 "$OUT/assign_trace.log"; exit 1; }
find "$OUT" -name "*.csv" | sort
