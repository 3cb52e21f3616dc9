set -e
mkdir -p gpurun_out/s6
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_kmeans.py tests/test_gpu_configs.py -k "bf16" > gpurun_out/s6/pytest.log 2>&1 || { tail -60 gpurun_out/s6/pytest.log; exit 1; }
tail -3 gpurun_out/s6/pytest.log
timeout -k 10 300 python tools/bench_assign.py > gpurun_out/s6/assign.json 2>gpurun_out/s6/assign.err || { tail -30 gpurun_out/s6/assign.err; exit 1; }
cat gpurun_out/s6/assign.json
timeout -k 10 60 rocprofv3 -L > gpurun_out/s6/counters.txt 2>&1 || true
grep -i "mfma\|MOPS" gpurun_out/s6/counters.txt | head -40 || true
