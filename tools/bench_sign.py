#!/usr/bin/env python3
"""BASELINE config 1 shape through the signed-payload path: 4096 x 1 KiB
payloads, hash-then-sign (types/signature.n2t:60-119) and validate
(:124-175) with the P-521 key of test/sign.c:27-45.

Reports, per stage: the GPU batch digest (net2_sha2_batch, host memory in
and out), ECDSA over the digests on host threads, and the batched
net2x_signature_create_batch / _validate_batch end to end; plus the same flow
with the oracle's CPU digests (the reference's per-payload SHA512 on one
core, test/sign.c's shape) as the baseline.  One JSON line per measurement.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


class Sig(ctypes.Structure):
    _fields_ = [("sign_alg", ctypes.c_char_p), ("hash_alg", ctypes.c_char_p),
                ("data", ctypes.c_void_p), ("datalen", ctypes.c_size_t)]


class IOV(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class SignReq(ctypes.Structure):
    """struct net2_sc_sign_req (include/net2/signed_carver.h)."""
    _fields_ = [("payload", ctypes.POINTER(IOV)), ("iovcnt", ctypes.c_size_t),
                ("hash_alg", ctypes.c_int), ("num_signatures", ctypes.c_uint32),
                ("signatures", ctypes.POINTER(ctypes.c_void_p)),
                ("out", ctypes.POINTER(Sig)), ("rc", ctypes.c_int)]


class HashReq(ctypes.Structure):
    """struct net2_sc_hash_req (include/net2/signed_carver.h)."""


HashReq._fields_ = [("payload", ctypes.c_void_p), ("iovcnt", ctypes.c_size_t),
                    ("hash_alg", ctypes.c_int),
                    ("done", ctypes.CFUNCTYPE(None, ctypes.POINTER(HashReq),
                                              ctypes.c_void_p)),
                    ("arg", ctypes.c_void_p), ("rc", ctypes.c_int),
                    ("digestlen", ctypes.c_uint32),
                    ("digest", ctypes.c_uint8 * 64)]


class ValReq(ctypes.Structure):
    """struct net2_sc_validate_req (include/net2/signed_carver.h)."""
    _fields_ = [("payload", ctypes.POINTER(IOV)), ("iovcnt", ctypes.c_size_t),
                ("sig", ctypes.POINTER(Sig)), ("sctx", ctypes.c_void_p),
                ("result", ctypes.c_int)]


def measure():
    """All stages in one dict (bench.py's extra_configs.c1)."""
    res = stages()
    out = {"metric": "signed payloads/s, 4096 x 1 KiB (BASELINE configs[0] shape), "
                     "hash-then-sign / validate with the P-521 key of test/sign.c",
           "workload": "4096 x 1 KiB payloads, SHA-512 sighash (the negotiated default) "
                       "and SHA-256, ECDSA-P521 on host threads",
           "stages": {}}
    for r in res:
        out["stages"][r["key"]] = {k: (round(v, 3) if isinstance(v, float) else v)
                                   for k, v in r.items() if k != "key"}
    return out


def stages():
    import ilias_net2_amd._lib as L
    from oracle import oracle
    import synth
    L.lib()
    S = ctypes.CDLL(os.path.join(ROOT, "ilias_net2_amd", "libnet2_sign.so"))
    S.net2x_signctx_privnew.restype = ctypes.c_void_p
    S.net2x_signctx_pubnew.restype = ctypes.c_void_p
    S.net2x_signctx_maxmsglen.restype = ctypes.c_size_t
    S.net2x_signctx_maxmsglen.argtypes = [ctypes.c_void_p]
    S.net2x_signature_deinit.restype = None
    keys = [open(os.path.join(ROOT, "tests", "golden", "keys", f), "rb").read()
            for f in ("ecdsa_p521_priv.pem", "ecdsa_p521_pub.pem")]
    priv = ctypes.c_void_p(S.net2x_signctx_privnew(0, keys[0], len(keys[0])))
    pub = ctypes.c_void_p(S.net2x_signctx_pubnew(0, keys[1], len(keys[1])))
    assert priv and pub
    n, length = 4096, 1024
    threads = min(16, len(os.sched_getaffinity(0)))
    data = synth.fixed_batch(1, n, length)
    offs = (np.arange(n, dtype=np.uint64) * length)
    lens = np.full(n, length, dtype=np.uint32)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    res = []

    def timeit(fn, reps=3):
        fn()
        best = 1e9
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t)
        return best

    for alg, name in ((3, "SHA512"), (1, "SHA256")):
        dig = np.empty((n, 64 if alg == 3 else 32), dtype=np.uint8)
        t = timeit(lambda: L.check(L.lib().net2_sha2_batch(
            alg, ptr(data), ptr(offs), ptr(lens), 0, 0, n, ptr(dig), 1)))
        res.append({"key": f"gpu_digest_{name.lower()}",
                     "stage": f"GPU digest {name} (net2_sha2_batch, host mem, 1 GPU)",
                    "payloads_per_s": n / t, "ms": t * 1e3})
        t = timeit(lambda: oracle.batch(alg, data, stride=length, length=length,
                                        n=n, nthreads=1))
        res.append({"key": f"cpu_digest_{name.lower()}_1core",
                    "stage": f"CPU digest {name} (oracle, 1 core = test/sign.c shape)",
                    "payloads_per_s": n / t, "ms": t * 1e3})
    sigs = (Sig * n)()
    valid = (ctypes.c_int * n)()

    def create():
        rc = S.net2x_signature_create_batch(sigs, ptr(data), ptr(offs), ptr(lens),
                                           ctypes.c_size_t(n), 3, priv, threads)
        assert rc == 0, rc

    def validate():
        rc = S.net2x_signature_validate_batch(sigs, ptr(data), ptr(offs), ptr(lens),
                                             ctypes.c_size_t(n), pub, valid, threads)
        assert rc == 0, rc

    def free_all():
        for i in range(n):
            S.net2x_signature_deinit(ctypes.byref(sigs[i]))

    create()
    t_c = 1e9
    for _ in range(2):
        free_all()
        t0 = time.perf_counter()
        create()
        t_c = min(t_c, time.perf_counter() - t0)
    t_v = timeit(validate, reps=2)
    assert all(v == 1 for v in valid)
    res.append({"key": "signature_create_batch",
                "stage": f"net2x_signature_create_batch SHA512+ECDSA-P521, {threads} threads",
                "payloads_per_s": n / t_c, "ms": t_c * 1e3})
    res.append({"key": "signature_validate_batch",
                "stage": f"net2x_signature_validate_batch SHA512+ECDSA-P521, {threads} threads",
                "payloads_per_s": n / t_v, "ms": t_v * 1e3})
    free_all()

    # the signed carver's signature step, one tick for all 4096 carvers
    # (src/signed_carver.c:407-432 batched; net2/signed_carver.h)
    iovs = (IOV * n)()
    for i in range(n):
        iovs[i].base = data.ctypes.data + i * length
        iovs[i].len = length
    ctxs = (ctypes.c_void_p * 1)(priv.value)
    reqs = (SignReq * n)()
    outs = (Sig * n)()
    for i in range(n):
        reqs[i].payload = ctypes.pointer(iovs[i])
        reqs[i].iovcnt = 1
        reqs[i].hash_alg = 3
        reqs[i].num_signatures = 1
        reqs[i].signatures = ctxs
        reqs[i].out = ctypes.pointer(outs[i])
    vreqs = (ValReq * n)()
    for i in range(n):
        vreqs[i].payload = ctypes.pointer(iovs[i])
        vreqs[i].iovcnt = 1
        vreqs[i].sig = ctypes.pointer(outs[i])
        vreqs[i].sctx = pub.value

    def sign_tick():
        for i in range(n):
            S.net2x_signature_deinit(ctypes.byref(outs[i]))
        rc = S.net2_signed_carver_sign_tick(reqs, ctypes.c_size_t(n), threads)
        assert rc == 0, rc

    def validate_tick():
        rc = S.net2_signed_combiner_validate_tick(vreqs, ctypes.c_size_t(n), threads)
        assert rc == 0, rc
    t_st = timeit(sign_tick, reps=2)
    assert all(reqs[i].rc == 0 for i in range(n))
    t_vt = timeit(validate_tick, reps=2)
    assert all(vreqs[i].result == 0 for i in range(n))
    res.append({"key": "signed_carver_sign_tick",
                "stage": f"net2_signed_carver_sign_tick: {n} carvers x 1 SHA512+ECDSA-P521 signature, one tick, {threads} threads",
                "payloads_per_s": n / t_st, "ms": t_st * 1e3})
    res.append({"key": "signed_combiner_validate_tick",
                "stage": f"net2_signed_combiner_validate_tick: {n} checks, one tick, {threads} threads",
                "payloads_per_s": n / t_vt, "ms": t_vt * 1e3})
    for i in range(n):
        S.net2x_signature_deinit(ctypes.byref(outs[i]))

    # the hash-only tick the reference's own sign layer binds to
    # (net2_sc_hash_req; the callbacks, here none, would run its ECDSA):
    # 4096 payloads' SHA-512 digests, one GPU batch
    hreqs = (HashReq * n)()
    for i in range(n):
        hreqs[i].payload = ctypes.addressof(iovs[i])
        hreqs[i].iovcnt = 1
        hreqs[i].hash_alg = 3

    def hash_tick():
        rc = S.net2_sc_hash_tick(hreqs, ctypes.c_size_t(n), threads)
        assert rc == 0, rc
    t_ht = timeit(hash_tick)
    want = oracle.batch(3, data, stride=length, length=length, n=n)
    assert all(bytes(hreqs[i].digest) == want[i].tobytes() for i in range(0, n, 97))
    res.append({"key": "sc_hash_tick",
                "stage": f"net2_sc_hash_tick: {n} x 1 KiB SHA512 digests, one tick (the "
                         "reference binding's hash step; its ECDSA runs in the callbacks)",
                "payloads_per_s": n / t_ht, "ms": t_ht * 1e3})
    return res


def main():
    for r in stages():
        r["config"] = "4096 x 1 KiB payloads (BASELINE configs[0] shape)"
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
