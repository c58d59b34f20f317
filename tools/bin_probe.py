#!/usr/bin/env python3
"""Where a one-pass binning launch spends its time: run with a library
built -DNET2_BIN_PROBE=1 (tools/build_ab.sh probe -DNET2_BIN_PROBE=1;
NET2_SHA2_LIB=tools/ab/probe.so), which has thread 0 of every workgroup
stamp the 100 MHz s_memrealtime clock at eight points of
bin_onepass_kernel into the workspace's spare words.  Prints, per point,
the min / median / max over workgroups in microseconds from the earliest
workgroup start, for the C3 mix and the burst-RX datagram mix.

  0 start (header read)   1 counted (LDS)      2 added to the histogram
  3 arrived               4 barrier decided    5 bin bases scanned
  6 perm written
"""
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
    hdr = L.net2_sha2_dev_var_workspace(0) // 4     # header + hist + cursor words
    nb = 2048
    for name, alg, choices in (("c3", 1, (64, 512, 1500)),
                               ("mtu_mix", 3, (0, 1, 17, 64, 136, 500, 1472))):
        n = 1 << 20
        lens = synth.mixed_lengths(7, n, choices=choices)
        data, offs = synth.packed(8, lens)
        d = torch.from_numpy(data).to(dev)
        o = torch.from_numpy(offs.astype(np.int64)).to(dev)
        ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
        ws = batch.var_workspace(n, dev)
        for _ in range(20):
            batch.digest_var(alg, d, o, ln, workspace=ws)
        torch.cuda.synchronize()
        base = 16 + 2 * nb + 2048          # after the histograms, barrier words
        st = ws.cpu().numpy().view(np.uint32)[base:base + 256 * 8]
        st = st.reshape(256, 8).astype(np.int64)
        st = st[st[:, 0] != 0]            # the grid's workgroups (G <= 256)
        st = (st - st[:, 0].min()) & 0xffffffff
        print(f"== {name}: {n} packets, {len(st)} workgroups (us from first start)")
        names = ["start", "counted", "hist added", "arrived", "decided",
                 "bases", "perm written"]
        for p in range(7):
            c = st[:, p] / 100.0
            print(f"  {p} {names[p]:13s} min {c.min():7.2f}  med {np.median(c):7.2f}"
                  f"  max {c.max():7.2f}")
        last = int(np.argmax(st[:, 3]))
        print(f"  last arriver: workgroup {last}, its stamps "
              f"{[round(float(v) / 100, 2) for v in st[last, :7]]}")
        assert hdr >= 16


if __name__ == "__main__":
    main()
