#!/usr/bin/env python3
"""Per-packet overhead of the variable-length kernels: one length per batch
(so the binned order changes nothing), hashed binned (perm -> offsets/lens,
plus the binning launches) and unbinned (offsets/lens by lane), SHA-512 and
HMAC-SHA512; HIP events over 50 launches each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from ilias_net2_amd import batch  # noqa: E402


def run(alg, ln, binned, n=1 << 20):
    dev = torch.device("cuda:0")
    lens = torch.full((n,), ln, dtype=torch.int32, device=dev)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * ln
    data = torch.randint(0, 256, (n * ln,), dtype=torch.uint8, device=dev)
    out = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    ws = batch.var_workspace(n, dev)
    key = bytes(range(64))

    def step():
        if alg >= 4:
            batch.hmac_dev(alg, key, data, offsets=offs, lens=lens, out=out,
                           workspace=ws, binned=binned)
        else:
            batch.digest_var(alg, data, offs, lens, out=out, workspace=ws, binned=binned)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        step()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 50 * 1e3


if __name__ == "__main__":
    for alg in (3, 6):
        for ln in (64, 512, 1428):
            tb, tu = run(alg, ln, True), run(alg, ln, False)
            print(f"alg {alg} len {ln:5d}: binned {tb:8.1f} us  unbinned {tu:8.1f} us  "
                  f"diff {tb - tu:6.1f} us", flush=True)
