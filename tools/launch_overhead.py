#!/usr/bin/env python3
"""Fixed cost per launch of the fixed-length kernels: time back-to-back
launches over n = 128 K ... 4 M packets of 1 KiB and fit t(n) = a + b n.
`a` is what a launch costs beyond its packets' share of the issue-bound
steady state (ramp-up, drain, launch gap); b * 1 M is the steady-state
time of a 1 M-packet batch.

  python tools/launch_overhead.py [--alg 1] [--reps 40]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from ilias_net2_amd import batch
    ap = argparse.ArgumentParser()
    ap.add_argument("--alg", type=int, default=1)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--sizes", default="131072,262144,524288,1048576,2097152,4194304")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    sizes = [int(x) for x in a.sizes.split(",")]
    nmax = max(sizes)
    data = torch.randint(0, 256, (nmax * 1024,), dtype=torch.uint8, device=dev)
    dl = 32 if a.alg == 1 else 64
    out = torch.empty((nmax * dl,), dtype=torch.uint8, device=dev)
    rows = []
    for alt in range(2):
        for n in sizes:
            o = out[:n * dl].view(n, dl)
            for _ in range(10):
                batch.digest_fixed(a.alg, data, 1024, 1024, n, out=o)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                batch.digest_fixed(a.alg, data, 1024, 1024, n, out=o)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            rows.append((n, ms))
            print(f"alt={alt} n={n} ms_per_launch={ms:.4f} ns_per_packet={ms * 1e6 / n:.3f}",
                  flush=True)
    x = np.array([r[0] for r in rows], dtype=np.float64)
    y = np.array([r[1] for r in rows], dtype=np.float64)
    b, c = np.polyfit(x, y, 1)
    print(f"fit: t(n) = {c * 1e3:.2f} us + n * {b * 1e6:.4f} ns; "
          f"1 M packets steady state {b * (1 << 20):.4f} ms, fixed cost "
          f"{c * 1e3:.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
