#!/usr/bin/env python3
"""Forged barrier words (tests/test_gpu_binning.py scenario 2) repeated:
how many launches abort, with the library NET2_SHA2_LIB points at.  A
measurement aid for the binning's fallback accounting."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import synth
    from ilias_net2_amd import _lib, batch
    L = _lib.lib()
    dev = torch.device("cuda:0")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lens = synth.mixed_lengths(3, n)
    data, offs = synth.packed(680, lens)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    ws = batch.var_workspace(n, dev)
    ctl0 = 16 + 2 * 2048
    G = (n + 4095) // 4096
    ref = batch.digest_var(1, d, o, ln, workspace=ws).cpu()
    for _ in range(reps):
        torch.cuda.synchronize()
        base = ctl0 + (int(ws[2].item()) & 1) * 1024
        ws[base + 512] = min(G, 16) - 1
        ws[base + 0] = (G + 15) // 16 - 1
        got = batch.digest_var(1, d, o, ln, workspace=ws)
        assert torch.equal(got.cpu(), ref)
        got = batch.digest_var(1, d, o, ln, workspace=ws)
        assert torch.equal(got.cpu(), ref)
    torch.cuda.synchronize()
    print(os.path.basename(os.environ.get("NET2_SHA2_LIB", "default")), n, reps,
          _lib.workspace_stats(ws.data_ptr(), ws.numel() * ws.element_size()))


if __name__ == "__main__":
    main()
