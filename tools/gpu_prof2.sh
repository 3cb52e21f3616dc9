#!/bin/bash
set -e
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 300 python tools/prof_kmeans.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o km -- python3 tools/prof_kmeans.py > gpurun_out/prof2.log 2>&1
