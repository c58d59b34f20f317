#!/usr/bin/env python3
"""End-to-end rates of net2_sha2_batch (host memory -> GPU -> host) for the
host layouts a caller can hand it: 1 M x 1 KiB fixed-stride packets from
pageable and from pinned memory, and 1 M x {64, 512, 1500} B packed
datagrams from pageable memory.  Best of 3 after a warm-up call."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402  (load torch's HIP runtime first)
import synth  # noqa: E402
from ilias_net2_amd import batch  # noqa: E402


def best(f):
    f()
    b = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        f()
        b = min(b, time.perf_counter() - t0)
    return b


n = 1 << 20
fixed = synth.fixed_batch(2, n, 1024)
t = best(lambda: batch.digest_host(1, fixed, stride=1024, length=1024, n=n, max_devices=1))
print(f"fixed 1 KiB, pageable: {n / t / 1e6:.1f} M digests/s, {n * 1024 / t / 1e9:.2f} GB/s", flush=True)
pinned = torch.from_numpy(fixed).pin_memory().numpy()
t = best(lambda: batch.digest_host(1, pinned, stride=1024, length=1024, n=n, max_devices=1))
print(f"fixed 1 KiB, pinned:   {n / t / 1e6:.1f} M digests/s, {n * 1024 / t / 1e9:.2f} GB/s", flush=True)
lens = synth.mixed_lengths(3, n)
data, offs = synth.packed(4, lens)
t = best(lambda: batch.digest_host(1, data, offsets=offs, lens=lens, max_devices=1))
print(f"mixed datagrams, pageable: {n / t / 1e6:.1f} M datagrams/s, {int(lens.sum()) / t / 1e9:.2f} GB/s", flush=True)
