#!/usr/bin/env python3
"""Latency of the single-message path (net2_hashctx_hashiov through the
ilias::hash mirror): one 1 KiB SHA-256 / one 1 KiB HMAC-SHA512 per call,
host memory in and out, median of 2,000 calls."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
from ilias_net2_amd import hash as h  # noqa: E402

msg = bytes(range(256)) * 4
for name, fac, key in (("SHA256", h.sha256(), b""),
                       ("HMAC-SHA512", h.hmac_sha512(), bytes(64))):
    fac.run(key, msg)
    ts = []
    for _ in range(2000):
        t0 = time.perf_counter()
        fac.run(key, msg)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"{name} 1 KiB single message: median {ts[1000] * 1e6:.1f} us, "
          f"p99 {ts[1980] * 1e6:.1f} us", flush=True)
