#!/bin/bash
# k-means++ changes: micro timing (fused path, and the LDS fold for comparison), then the kpp /
# MiniBatch parity tests. Each GPU step time-limited; the first failure ends the script.
set -e
OUT=gpurun_out/${1:-kpp}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/micro_kpp.py > "$OUT/micro.log" 2>&1 || { tail -20 "$OUT/micro.log"; exit 1; }
cat "$OUT/micro.log"
GDD_KPP_LDS_FOLD=1 timeout -k 10 200 python -u tools/micro_kpp.py > "$OUT/micro_lds.log" 2>&1 || { tail -20 "$OUT/micro_lds.log"; exit 1; }
cat "$OUT/micro_lds.log"
PYT="python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu"
timeout -k 10 600 $PYT tests/test_gpu_kpp.py tests/test_gpu_golden.py tests/test_gpu_kmeans.py tests/test_gpu_edge.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
