#!/usr/bin/env python3
"""Per-block cost of the variable-length kernels by packet length:
1 M packed packets of one length (then the C3 mix), binned,
device-resident; kernel time from HIP events over 50 launches.  Prints
ns per compression (blocks incl. padding, and the HMAC outer block) --
equal numbers mean every bin runs at the same issue rate, so a mix's gap to
its floor is not one bin's; a mix slower than its bins' average is the
cost of the mix itself (e.g. waves of one workgroup running different
code paths).
  python tools/var_bins.py [--alg 1|3|4|6] [--lens 64,512,1500 ...]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from ilias_net2_amd import batch  # noqa: E402

BLOCK = {1: 64, 3: 128, 4: 64, 6: 128}
LENB = {1: 8, 3: 16, 4: 8, 6: 16}
DLEN = {1: 32, 3: 64, 4: 32, 6: 64}


def run(alg, choice, n=1 << 20):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    ch = torch.tensor(choice, dtype=torch.int64, device=dev)
    lens = ch[torch.randint(0, len(choice), (n,), device=dev, generator=g)]
    offs = torch.zeros(n, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)[:-1]
    data = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8, device=dev, generator=g)
    l32 = lens.to(torch.int32)
    out = torch.empty((n, DLEN[alg]), dtype=torch.uint8, device=dev)
    ws = batch.var_workspace(n, dev)
    B, hm = BLOCK[alg], alg >= 4
    # inner blocks from the IV (or the ipad midstate) incl. padding, + outer
    nblk = int(((lens + LENB[alg] + 1 + B - 1) // B).sum()) + (n if hm else 0)
    key = bytes(range(DLEN[alg]))

    def step():
        if hm:
            batch.hmac_dev(alg, key, data, offsets=offs, lens=l32, out=out, workspace=ws)
        else:
            batch.digest_var(alg, data, offs, l32, out=out, workspace=ws)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        step()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 50
    print(f"alg {alg} {str(choice):18s} {ms * 1e3:8.1f} us/launch  {nblk / 1e6:6.2f} M blocks  "
          f"{ms * 1e6 / nblk * 1024:7.1f} SIMD-ns per block (x1024 SIMDs)", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--alg", type=int, default=1, choices=sorted(BLOCK))
    ap.add_argument("--lens", nargs="*", default=["64", "512", "1500", "64,512,1500", "1024"])
    args = ap.parse_args()
    for c in args.lens:
        run(args.alg, [int(x) for x in c.split(",")])
