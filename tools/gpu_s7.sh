set -e
mkdir -p gpurun_out/s7
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 500 $PYT tests/test_gpu_kpp.py tests/test_gpu_configs.py tests/test_gpu_kmeans.py tests/test_gpu_edge.py tests/test_gpu_golden.py tests/test_gpu_recsys.py > gpurun_out/s7/pytest.log 2>&1 || { tail -60 gpurun_out/s7/pytest.log; exit 1; }
tail -3 gpurun_out/s7/pytest.log
timeout -k 10 300 python tools/prof_lloyd.py > gpurun_out/s7/lloyd.log 2>&1 || { tail -30 gpurun_out/s7/lloyd.log; exit 1; }
grep KMeans gpurun_out/s7/lloyd.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_assign" --output-format csv -d gpurun_out/s7/pmc_mfma -o assign -- python3 tools/bench_assign.py > gpurun_out/s7/pmc_mfma.log 2>&1 || { tail -20 gpurun_out/s7/pmc_mfma.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s7/assign_trace -o assign -- python3 tools/bench_assign.py > gpurun_out/s7/assign_trace.log 2>&1 || { tail -20 gpurun_out/s7/assign_trace.log; exit 1; }
ls gpurun_out/s7/pmc_mfma gpurun_out/s7/assign_trace
