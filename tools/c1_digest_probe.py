#!/usr/bin/env python3
"""C1's GPU digest stage alone: 4096 x 1 KiB from host memory through
net2_sha2_batch (variable layout, one GPU), SHA-512 and SHA-256; min and
median of 30 calls after a warm-up.  NET2_SHA2_NUMA / NET2_SHA2_LIB select
the variant."""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (loads torch's HIP runtime first)
from ilias_net2_amd import _lib as L  # noqa: E402

n, length = 4096, 1024
data = np.random.default_rng(1).integers(0, 256, n * length, dtype=np.uint8)
offs = np.arange(n, dtype=np.uint64) * length
lens = np.full(n, length, dtype=np.uint32)


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


for alg in (3, 1, 3, 1):
    dig = np.empty((n, 64), dtype=np.uint8)
    f = lambda: L.check(L.lib().net2_sha2_batch(  # noqa: E731
        alg, ptr(data), ptr(offs), ptr(lens), 0, 0, n, ptr(dig), 1))
    f()
    ts = []
    for _ in range(30):
        t = time.perf_counter()
        f()
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"NUMA={os.environ.get('NET2_SHA2_NUMA', '1')} alg {alg}: min {min(ts):.3f} "
          f"median {statistics.median(ts):.3f} ms", flush=True)
