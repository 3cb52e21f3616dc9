#!/bin/bash
# Config-shape end-to-end measurements: arxiv phases, products (config 5), Reddit inductive (config 3).
set -e
OUT=gpurun_out/${1:-shapes}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/phase_times.py > "$OUT/phases.log" 2>&1 || { tail -20 "$OUT/phases.log"; exit 1; }
grep rep "$OUT/phases.log" | tail -2
timeout -k 10 500 python -u tools/bench_products.py > "$OUT/products.log" 2>&1 || { tail -20 "$OUT/products.log"; exit 1; }
tail -1 "$OUT/products.log"
timeout -k 10 400 python -u tools/bench_induct.py > "$OUT/induct.log" 2>&1 || { tail -20 "$OUT/induct.log"; exit 1; }
tail -1 "$OUT/induct.log"
