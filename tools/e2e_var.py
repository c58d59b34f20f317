#!/usr/bin/env python3
"""End-to-end rate of the variable-layout host path (net2_sha2_batch with
offsets/lengths): 1 M x {64, 512, 1500} B datagrams back to back in ordinary
(pageable) host memory -> staging gather -> H2D -> binned kernel -> D2H, or
(argument "pinned") in page-locked memory, copied as they lie."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (load torch's HIP runtime first)
import synth  # noqa: E402
from ilias_net2_amd import batch  # noqa: E402

lens = synth.mixed_lengths(3, 1 << 20)
data, offs = synth.packed(4, lens)
memory = sys.argv[1] if len(sys.argv) > 1 else "pageable"
if memory == "pinned":      # a page-locked receive arena: DMA'd as it lies
    data = torch.from_numpy(data).pin_memory().numpy()
batch.digest_host(1, data, offsets=offs, lens=lens, max_devices=1)   # warm-up
best = 1e9
for _ in range(3):
    t0 = time.perf_counter()
    batch.digest_host(1, data, offsets=offs, lens=lens, max_devices=1)
    best = min(best, time.perf_counter() - t0)
print(f"var e2e ({memory}): {len(lens) / best / 1e6:.1f} M datagrams/s, "
      f"{int(lens.sum()) / best / 1e9:.2f} GB/s of payload", flush=True)
