#!/usr/bin/env python3
"""C3 read-traffic diagnosis: the same 1 M x {64, 512, 1500} B batch hashed
(length-binned) from four layouts -- packed back to back (BASELINE config
C3), every packet start rounded up to 16 bytes (what net2_sha2_batch's
packer does), to 128 bytes (no two packets share a line, and every block
pair of a packet is line-aligned), and packed but hashed unbinned (memory
order) -- 5 launches each, in that order.  Run under `rocprofv3 --pmc
FETCH_SIZE` or `--pmc TCC_EA0_RDREQ ...`; the per-dispatch counts of
var_kernel then separate the sources of re-read lines."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402
from ilias_net2_amd import batch  # noqa: E402

dev = torch.device("cuda:0")
lens = synth.mixed_lengths(3, 1 << 20)
for align, binned in ((1, True), (16, True), (128, True), (1, False)):
    data, offs = synth.packed(4, lens, align=align)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    for _ in range(5):
        batch.digest_var(1, d, o, ln, binned=binned)
    torch.cuda.synchronize()
    print(f"align={align} binned={binned} payload={int(lens.sum())}", flush=True)
