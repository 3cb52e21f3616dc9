set -e
mkdir -p gpurun_out/s3
export TMPDIR=/tmp
timeout -k 10 300 python tools/prof_lloyd.py > gpurun_out/s3/lloyd.log 2>&1 || { tail -30 gpurun_out/s3/lloyd.log; exit 1; }
cat gpurun_out/s3/lloyd.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3/trace -o lloyd -- python3 tools/prof_lloyd.py > gpurun_out/s3/trace.log 2>&1 || { tail -30 gpurun_out/s3/trace.log; exit 1; }
