set -e
mkdir -p gpurun_out/s5
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_agent.py > gpurun_out/s5/pytest_agent.log 2>&1 || { tail -60 gpurun_out/s5/pytest_agent.log; exit 1; }
tail -3 gpurun_out/s5/pytest_agent.log
timeout -k 10 900 $PYT tests > gpurun_out/s5/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/s5/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/s5/pytest_gpu.log
timeout -k 10 600 python -u -m gdd.train_clustgdd_transduct --dataset ogbn-arxiv --reduction_rate 0.005 --prop_num 18 --postprop_num 10 --alpha 0.91 --predropout 0.6 --sp_ratio 0.1 --preep 1000 --postep 1000 --frcoe 1.9 --predcoe 0.025 --json gpurun_out/s5/arxiv_accuracy.json > gpurun_out/s5/arxiv_agent.log 2>&1 || { tail -30 gpurun_out/s5/arxiv_agent.log; exit 1; }
tail -6 gpurun_out/s5/arxiv_agent.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s5/lloyd -o lloyd -- python3 tools/prof_lloyd.py > gpurun_out/s5/lloyd.log 2>&1 || { tail -30 gpurun_out/s5/lloyd.log; exit 1; }
grep KMeans gpurun_out/s5/lloyd.log
