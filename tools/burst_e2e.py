#!/usr/bin/env python3
"""The host-memory burst rates of bench.py's extra_configs (burst_rx_e2e /
burst_tx_e2e) on their own, for the per-chunk host timings
(NET2_SHA2_DEBUG_TIMING=1 prints pack / wait / finish per chunk to stderr).
  python tools/burst_e2e.py [rx|tx] [pinned|pageable]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "tx"
memory = sys.argv[2] if len(sys.argv) > 2 else "pinned"
print(json.dumps(bench.burst_e2e_rate(kind, steps=4, warmup=1, memory=memory)))
