#!/usr/bin/env python3
"""net2_sha2_batch end to end (pinned in, pinned out, one GPU) by batch size:
1 KiB packets, 16 K .. 1 M of them; best of 5 after a warm-up."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from ilias_net2_amd import _lib  # noqa: E402

L = _lib.lib()
N = 1 << 20
src = torch.randint(0, 256, (N * 1024,), dtype=torch.uint8).pin_memory()
out = torch.empty((N, 32), dtype=torch.uint8).pin_memory()
for n in (1 << 14, 1 << 16, 1 << 17, 1 << 18, 1 << 20):
    f = lambda: _lib.check(L.net2_sha2_batch(1, src.data_ptr(), None, None, 1024, 1024, n,  # noqa: E731
                                             out.data_ptr(), 1))
    f()
    best = 1e9
    for _ in range(5):
        t = time.perf_counter()
        f()
        best = min(best, time.perf_counter() - t)
    print(f"{n:8d} x 1 KiB: {best * 1e3:8.3f} ms  {n / best / 1e6:6.1f} M/s  {n * 1024 / best / 1e9:6.2f} GB/s", flush=True)
