#!/bin/bash
# End-to-end drivers on the device: config 4 (distill_recsys at the ML-1M shape) and the
# transductive agent at the ogbn-arxiv shape with main_transduct.sh's r=0.5% flags (accuracy + time).
set -e
OUT=gpurun_out/${1:-e2e}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/bench_recsys_e2e.py > "$OUT/recsys.log" 2>&1 || { tail -20 "$OUT/recsys.log"; exit 1; }
tail -1 "$OUT/recsys.log"
PYTHONPATH=graph-distillation-for-recommendation_amd timeout -k 10 600 python -u -m gdd.train_clustgdd_transduct --gpu_id 0 --dataset ogbn-arxiv \
  --reduction_rate 0.005 --prop_num 18 --postprop_num 10 --alpha 0.91 --predropout 0.6 \
  --sp_ratio 0.1 --preep 1000 --postep 1000 --frcoe 1.9 --predcoe 0.025 --save 1 \
  --json "$OUT/agent_arxiv.json" > "$OUT/agent_arxiv.log" 2>&1 || { tail -30 "$OUT/agent_arxiv.log"; exit 1; }
tail -12 "$OUT/agent_arxiv.log"
