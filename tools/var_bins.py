#!/usr/bin/env python3
"""Per-block cost of the SHA-256 variable-length kernel by packet length:
1 M packed packets of one length (64, 512, 1500 B, then the C3 mix), binned,
device-resident; kernel time from HIP events over 50 launches.  Prints
ns per compression (blocks incl. padding) -- equal numbers mean every bin
runs at the same issue rate, so C3's gap to its floor is not one bin's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from ilias_net2_amd import batch  # noqa: E402


def run(choice, n=1 << 20):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    ch = torch.tensor(choice, dtype=torch.int64, device=dev)
    lens = ch[torch.randint(0, len(choice), (n,), device=dev, generator=g)]
    offs = torch.zeros(n, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)[:-1]
    data = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8, device=dev, generator=g)
    l32 = lens.to(torch.int32)
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    ws = batch.var_workspace(n, dev)
    nblk = int(((lens + 8 + 1 + 63) // 64).sum())
    for _ in range(20):
        batch.digest_var(1, data, offs, l32, out=out, workspace=ws)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        batch.digest_var(1, data, offs, l32, out=out, workspace=ws)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 50
    print(f"{str(choice):18s} {ms * 1e3:8.1f} us/launch  {nblk / 1e6:6.2f} M blocks  "
          f"{ms * 1e6 / nblk * 1024:7.1f} SIMD-ns per block (x1024 SIMDs)", flush=True)


if __name__ == "__main__":
    for c in ([64], [512], [1500], [64, 512, 1500], [1024]):
        run(c)
