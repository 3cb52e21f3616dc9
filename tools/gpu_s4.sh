set -e
mkdir -p gpurun_out/s4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu_kmeans.py -k "center_columns" > gpurun_out/s4/pytest.log 2>&1 || { tail -40 gpurun_out/s4/pytest.log; exit 1; }
tail -2 gpurun_out/s4/pytest.log
timeout -k 10 300 python tools/micro_fold.py > gpurun_out/s4/fold.log 2>&1 || { tail -30 gpurun_out/s4/fold.log; exit 1; }
cat gpurun_out/s4/fold.log
timeout -k 10 300 python tools/prof_lloyd.py > gpurun_out/s4/lloyd.log 2>&1 || { tail -30 gpurun_out/s4/lloyd.log; exit 1; }
cat gpurun_out/s4/lloyd.log
