#!/usr/bin/env python3
"""Cost of the packet-burst RX path (net2_packet_decode_burst, HMAC-SHA512
+ 16-byte IVs) by datagram length: 1 M wire datagrams of one length, then
the {136, 584, 1500} B mix of bench.py's burst_rx config, encoded by
net2_packet_encode_burst first so every datagram verifies.  Run it under
`rocprofv3 --kernel-trace --stats`, one length set per process
(tools/gpu_burst_bins.sh), for the per-kernel split; it prints the compressions
per launch (inner blocks after the ipad midstate, incl. padding, + the outer
block) so the HMAC kernel's time per compression can be set beside the
variable-length kernels' (tools/var_bins.py).
  python tools/burst_bins.py --lens 136|584|1500|136,584,1500"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from ilias_net2_amd import _lib  # noqa: E402

ALG = 6			# HMAC-SHA512, the negotiated per-datagram hash
KEY = bytes(range(64))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="136,584,1500")
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    choice = [int(x) for x in a.lens.split(",")]
    n = a.n
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    ch = torch.tensor(choice, dtype=torch.int64, device=dev)
    lens = ch[torch.randint(0, len(choice), (n,), device=dev, generator=g)]
    offs = torch.zeros(n, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)[:-1]
    data = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8,
                         device=dev, generator=g)
    l32 = lens.to(torch.int32)
    seq = torch.arange(n, dtype=torch.int32, device=dev)
    flags = torch.full((n,), 3, dtype=torch.int32, device=dev)  # SIGNED|ENCRYPTED
    iv = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    oseq = torch.empty(n, dtype=torch.int32, device=dev)
    ofl = torch.empty(n, dtype=torch.int32, device=dev)
    res = torch.empty(n, dtype=torch.uint8, device=dev)
    L = _lib.lib()
    ws = torch.empty(L.net2_packet_burst_workspace(n), dtype=torch.uint8,
                     device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(L.net2_packet_encode_burst(
        ALG, KEY, len(KEY), 1, seq.data_ptr(), flags.data_ptr(),
        data.data_ptr(), offs.data_ptr(), l32.data_ptr(), n, res.data_ptr(),
        ws.data_ptr(), ws.numel(), s))
    torch.cuda.synchronize()
    assert int((res != 0).sum()) == 0, "encode failed"

    def step():
        _lib.check(L.net2_packet_decode_burst(
            ALG, KEY, len(KEY), 1, 16, data.data_ptr(), offs.data_ptr(),
            l32.data_ptr(), n, res.data_ptr(), iv.data_ptr(), oseq.data_ptr(),
            ofl.data_ptr(), ws.data_ptr(), ws.numel(), s))
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    assert int((res != 0).sum()) == 0, "decode failed"
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.steps):
        step()
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / a.steps
    m = lens - 8 - 64			# payload after header and hash field
    comp = int(((m + 17 + 127) // 128).sum()) + n
    print(f"lens {a.lens:14s} {ms * 1e3:8.1f} us/step  {comp / 1e6:6.2f} M "
          f"compressions  {ms * 1e6 / comp * 1024:7.1f} SIMD-ns per compression "
          f"(whole step, x1024 SIMDs)", flush=True)


if __name__ == "__main__":
    main()
