#!/usr/bin/env python3
"""Single-payload latency at the reference's limits, and where batching
starts to pay (ADVICE round 3 on long messages).

The reference hashes one signed payload per call, up to 65,536 bytes
(src/carver.c:150,161; types/signature.n2t:92).  On the GPU one message is
one wave's serial chain of compressions, so a lone call is latency-bound;
many payloads per call are the throughput path.  Measured here, one JSON
line per row:

  single      net2_hashctx_hashiov of one 65,536-B SHA-512 payload (and one
              1 KiB for scale), median of 30 calls, against the oracle's
              digest of the same payload on one CPU core;
  tick1       a one-payload net2_signed_carver_sign_tick (hash + one
              ECDSA-P521 signature) and a one-payload net2_sc_hash_tick;
  crossover   net2_sha2_batch (host memory in and out, this GPU) of k
              payloads of 1 KiB / 64 KiB against the oracle on 1 and 16
              threads, k = 1 .. 16,384: the smallest k at which the GPU wins;
  long        one 256 MiB SHA256Update and four 32 MiB hashiov calls (the
              64 MiB request pieces of NET2_SHA2_STREAM_CHUNK, staging kept
              between requests), MB/s.

Usage: python tools/latency_long.py [--skip-long] > gpurun_out/latency_long.jsonl
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def emit(d):
    print(json.dumps(d), flush=True)


def med(ts):
    ts = sorted(ts)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-long", action="store_true")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch first)
    import ilias_net2_amd._lib as L
    from ilias_net2_amd import hash as h
    from oracle import oracle
    import synth
    lib = L.lib()
    rng = np.random.default_rng(1)

    # ---- single payloads ------------------------------------------------
    for alg, name, n in ((3, "SHA512", 65536), (3, "SHA512", 1024),
                         (1, "SHA256", 65536)):
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        fac = {1: h.sha256(), 3: h.sha512()}[alg]
        assert fac.run(b"", m) == oracle.digest(alg, m)
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            fac.run(b"", m)
            ts.append(time.perf_counter() - t0)
        cs = []
        for _ in range(30):
            t0 = time.perf_counter()
            oracle.digest(alg, m)
            cs.append(time.perf_counter() - t0)
        emit({"row": "single", "alg": name, "payload_bytes": n,
              "gpu_hashiov_median_us": round(med(ts) * 1e6, 1),
              "gpu_hashiov_p90_us": round(sorted(ts)[26] * 1e6, 1),
              "cpu_oracle_1core_median_us": round(med(cs) * 1e6, 1),
              "gpu_over_cpu": round(med(ts) / med(cs), 2)})

    # ---- one-payload ticks ----------------------------------------------
    import bench_sign as bs
    HashReq = bs.HashReq
    S = ctypes.CDLL(os.path.join(ROOT, "ilias_net2_amd", "libnet2_sign.so"))
    S.net2x_signctx_privnew.restype = ctypes.c_void_p
    S.net2x_signature_deinit.restype = None
    key = open(os.path.join(ROOT, "tests", "golden", "keys",
                            "ecdsa_p521_priv.pem"), "rb").read()
    priv = ctypes.c_void_p(S.net2x_signctx_privnew(0, key, len(key)))
    assert priv
    m = rng.integers(0, 256, 65536, dtype=np.uint8)
    iov = (bs.IOV * 1)(bs.IOV(m.ctypes.data, 65536))
    ctxs = (ctypes.c_void_p * 1)(priv)
    sig = (bs.Sig * 1)()
    ts = []
    for r in range(11):
        req = (bs.SignReq * 1)(bs.SignReq(ctypes.cast(iov, ctypes.POINTER(bs.IOV)), 1,
                                          3, 1, ctxs, sig, 0))
        t0 = time.perf_counter()
        rc = S.net2_signed_carver_sign_tick(req, 1, 1)
        ts.append(time.perf_counter() - t0)
        assert rc == 0 and req[0].rc == 0
        S.net2x_signature_deinit(ctypes.byref(sig[0]))
    hs = []
    for r in range(11):
        hr = (HashReq * 1)()
        hr[0].payload = ctypes.addressof(iov)
        hr[0].iovcnt = 1
        hr[0].hash_alg = 3
        t0 = time.perf_counter()
        rc = S.net2_sc_hash_tick(hr, 1, 1)
        hs.append(time.perf_counter() - t0)
        assert rc == 0 and bytes(hr[0].digest) == oracle.digest(3, m.tobytes())
    emit({"row": "tick1", "payload_bytes": 65536, "alg": "SHA512",
          "sign_tick_median_us": round(med(ts) * 1e6, 1),
          "hash_tick_median_us": round(med(hs) * 1e6, 1),
          "note": "one carver, one ECDSA-P521 signature; the hash tick is the "
                  "net2_sc_hash_tick the reference binding uses (no callback)"})

    # ---- crossover ---------------------------------------------------------
    threads = min(16, len(os.sched_getaffinity(0)))
    for length in (1024, 65536):
        rows = []
        for k in (1, 4, 16, 64, 256, 1024, 4096, 16384):
            if k * length > (1 << 30):
                break
            data = synth.fixed_batch(3, k, length)
            host = torch.from_numpy(data)
            dig = np.empty((k, 64), dtype=np.uint8)
            call = lambda: L.check(lib.net2_sha2_batch(  # noqa: E731
                3, host.data_ptr(), None, None, length, length, k,
                dig.ctypes.data, 1))
            call()
            reps = 5 if k * length < (64 << 20) else 2
            g = []
            for _ in range(reps):
                t0 = time.perf_counter()
                call()
                g.append(time.perf_counter() - t0)
            want = oracle.batch(3, data, stride=length, length=length, n=k)
            assert np.array_equal(dig, want)
            c1 = []
            for _ in range(2):
                t0 = time.perf_counter()
                oracle.batch(3, data, stride=length, length=length, n=k, nthreads=1)
                c1.append(time.perf_counter() - t0)
            cn = []
            for _ in range(2):
                t0 = time.perf_counter()
                oracle.batch(3, data, stride=length, length=length, n=k,
                             nthreads=threads)
                cn.append(time.perf_counter() - t0)
            rows.append({"k": k, "gpu_ms": round(min(g) * 1e3, 3),
                         "cpu_1core_ms": round(min(c1) * 1e3, 3),
                         f"cpu_{threads}threads_ms": round(min(cn) * 1e3, 3)})
        win1 = next((r["k"] for r in rows if r["gpu_ms"] < r["cpu_1core_ms"]), None)
        winn = next((r["k"] for r in rows
                     if r["gpu_ms"] < r[f"cpu_{threads}threads_ms"]), None)
        emit({"row": "crossover", "alg": "SHA512", "payload_bytes": length,
              "entry": "net2_sha2_batch, host memory in and out, one GPU",
              "gpu_wins_vs_1core_from_k": win1,
              f"gpu_wins_vs_{threads}threads_from_k": winn, "rows": rows})

    # ---- long messages -----------------------------------------------------
    if args.skip_long:
        return
    big = torch.randint(0, 256, (256 << 20,), dtype=torch.uint8)
    ctx = ctypes.create_string_buffer(208)
    out = ctypes.create_string_buffer(64)
    t0 = time.perf_counter()
    lib.SHA256Init(ctx)
    lib.SHA256Update(ctx, ctypes.c_void_p(big.data_ptr()), ctypes.c_size_t(big.numel()))
    lib.SHA256Final(out, ctx)
    el = time.perf_counter() - t0
    emit({"row": "long", "what": "SHA256Update of 256 MiB (four 64 MiB requests)",
          "s": round(el, 3), "MBps": round(big.numel() / el / 1e6, 2)})
    m32 = big[:32 << 20]
    iv = (L.IOVec * 1)(L.IOVec(ctypes.c_void_p(m32.data_ptr()), m32.numel()))
    d = ctypes.create_string_buffer(64)
    ts = []
    for _ in range(4):
        t0 = time.perf_counter()
        L.check(lib.net2_hashctx_hashiov(1, None, 0, iv, 1, d, 64))
        ts.append(time.perf_counter() - t0)
    d = d.raw[:32]
    emit({"row": "long", "what": "4 x net2_hashctx_hashiov of 32 MiB SHA-256",
          "s_each": [round(t, 3) for t in ts],
          "MBps": round(4 * m32.numel() / sum(ts) / 1e6, 2), "digest": d.hex()[:16]})


if __name__ == "__main__":
    main()
