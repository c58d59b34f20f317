#!/usr/bin/env python3
"""Host packet bursts by burst size.

net2_packet_decode_burst_host / _encode_burst_host (HMAC-SHA512, 16-byte
IVs, wire datagrams of {136, 584, 1500} B, every one PH_SIGNED|PH_ENCRYPTED)
at n in {64, 256, 1024, 4096, 16 K, 64 K, 1 M} datagrams from pinned and
from pageable host memory, one GPU (max_devices 1): per-call latency (median
and best of the repetitions after a warm-up) and datagrams/s.  Beside each
size, the oracle's restatement of the same calls (oracle_packet_*_batch,
test infrastructure, here only as the CPU figure) on 1 and 16 threads.  One
JSON object per line; every GPU result is checked against the oracle once per
size.

  python tools/burst_sizes.py [--sizes 64,256,...] [--out FILE]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ilias_net2_amd import _lib  # noqa: E402
from oracle import oracle  # noqa: E402

SIZES = [64, 256, 1024, 4096, 16384, 65536, 1 << 20]
KEY = bytes(range(64))
ALG, IVLEN = 6, 16


def reps_for(n):
    return max(20, min(400, (1 << 22) // n))


def host(shape, dt, pinned):
    if pinned:
        t = torch.empty(shape, dtype={np.uint8: torch.uint8, np.uint32: torch.int32}[dt],
                        pin_memory=True)
        return t.numpy().view(dt)
    return np.empty(shape, dtype=dt)


def timed(fn, reps, budget_s=3.0):
    fn()
    fn()
    ts = []
    t_all = time.perf_counter()
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        if time.perf_counter() - t_all > budget_s and len(ts) >= 5:
            break
    return statistics.median(ts), min(ts), len(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default=",".join(map(str, SIZES)))
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-oracle", action="store_true")
    args = ap.parse_args()
    sizes = [int(s) for s in args.sizes.split(",")]
    L = _lib.lib()
    O = oracle.lib()
    p = lambda a: a.ctypes.data  # noqa: E731
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    sz, u32 = ctypes.c_size_t, ctypes.c_uint32
    out = open(args.out, "w") if args.out else None
    nmax = max(sizes)
    rng = np.random.default_rng(11)
    lens_all = rng.choice(np.array([136, 584, 1500], dtype=np.uint32), nmax)
    kb = ctypes.create_string_buffer(KEY, 64)
    keys = _lib.BurstRxKeys(ALG, ctypes.cast(kb, ctypes.c_void_p), 64, 1, None, 0, 0, 0, 0)
    cpu16 = min(16, len(os.sched_getaffinity(0)))
    for memory in ("pinned", "pageable"):
        pin = memory == "pinned"
        for n in sizes:
            lens = lens_all[:n].copy()
            offs = np.zeros(n, dtype=np.uint64)
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            total = int(lens.sum())
            data = host((total,), np.uint8, pin)
            data[:] = rng.integers(0, 256, total, dtype=np.uint8)
            seq = np.arange(n, dtype=np.uint32)
            flags = np.full(n, 3, dtype=np.uint32)
            res = host((n,), np.uint8, pin)
            iv = host((n, IVLEN), np.uint8, pin)
            oseq, ofl = host((n,), np.uint32, pin), host((n,), np.uint32, pin)

            def tx():
                _lib.check(L.net2_packet_encode_burst_host(
                    ALG, KEY, 64, 1, p(seq), p(flags), p(data), p(offs), p(lens), n,
                    p(res), 1), "encode_burst_host")

            def rx():
                _lib.check(L.net2_packet_decode_burst_host(
                    ctypes.byref(keys), IVLEN, p(data), p(offs), p(lens), n, p(res),
                    p(iv), p(oseq), p(ofl), 1), "decode_burst_host")
            # parity once per size: TX against the oracle, then RX
            o_res, o_sealed = oracle.packet_encode_batch(ALG, KEY, True, seq, flags, data,
                                                         offs, lens, nthreads=cpu16)
            tx()
            assert np.array_equal(res, o_res) and np.array_equal(data, o_sealed), (memory, n)
            want = oracle.packet_decode_batch(ALG, KEY, True, IVLEN, data, offs, lens,
                                              nthreads=cpu16)
            rx()
            assert np.array_equal(res, want[0]) and (res == 0).all(), (memory, n)
            assert np.array_equal(iv, want[1]) and np.array_equal(oseq, want[2]), (memory, n)
            reps = reps_for(n)
            for kind, fn in (("rx", rx), ("tx", tx)):
                med, best, k = timed(fn, reps)
                row = {"kind": kind, "memory": memory, "n": n, "bytes": total,
                       "reps": k, "median_us": round(med * 1e6, 1),
                       "best_us": round(best * 1e6, 1),
                       "datagrams_per_s": round(n / med, 1),
                       "us_per_datagram": round(med * 1e6 / n, 4),
                       "parity": "bit-exact vs oracle"}
                if pin and not args.no_oracle:
                    # the CPU restatement of the same call, same buffers
                    o_res = np.empty(n, dtype=np.uint8)
                    o_iv = np.empty((n, IVLEN), dtype=np.uint8)
                    o_sq = np.empty(n, dtype=np.uint32)
                    o_fl = np.empty(n, dtype=np.uint32)
                    scratch = np.array(data, copy=True)
                    for t in (1, cpu16):
                        if kind == "rx":
                            f = lambda t=t: O.oracle_packet_decode_batch(  # noqa: E731
                                ALG, KEY, sz(64), None, sz(0), 0, u32(0), u32(0), 1,
                                sz(IVLEN), vp(data), vp(offs), vp(lens), sz(n), vp(o_res),
                                vp(o_iv), vp(o_sq), vp(o_fl), t)
                        else:
                            f = lambda t=t: O.oracle_packet_encode_batch(  # noqa: E731
                                ALG, KEY, sz(64), 1, vp(seq), vp(flags), vp(scratch),
                                vp(offs), vp(lens), sz(n), vp(o_res), t)
                        m, _, _ = timed(f, max(5, min(reps, (1 << 18) // n)), budget_s=4.0)
                        row[f"oracle_{t}t_us"] = round(m * 1e6, 1)
                        row[f"oracle_{t}t_datagrams_per_s"] = round(n / m, 1)
                line = json.dumps(row)
                print(line, flush=True)
                if out:
                    out.write(line + "\n")
                    out.flush()
            del data, res, iv, oseq, ofl
    if out:
        out.close()


if __name__ == "__main__":
    main()
