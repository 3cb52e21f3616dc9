#!/usr/bin/env python3
"""Config 3's whole inductive pass once (bench.reddit_record, no CPU baseline), for a kernel trace:
rocprofv3 --kernel-trace --stats -- python3 tools/prof_reddit.py. Prints the record's phases."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import bench  # noqa: E402

rec = bench.reddit_record("cuda", False, reps=1)
print(json.dumps({"ms_total": rec.get("ms_total"), "phases_ms": rec.get("phases_ms")}))
