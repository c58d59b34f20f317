"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU oracle.

Loads oracle/liboracle_sha2.so (built from oracle/sha2_oracle.c by
oracle/Makefile), the clean-room restatement of the reference's src/sha2.c.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
always as the checker / CPU baseline, never as the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_sha2.so")

DIGEST_LEN = {1: 32, 2: 48, 3: 64, 4: 32, 5: 48, 6: 64}


class Ctx(ctypes.Structure):
    """oracle_sha2_ctx == the reference SHA2_CTX layout (208 bytes)."""
    _fields_ = [("st", ctypes.c_uint64 * 8), ("bits", ctypes.c_uint64 * 2),
                ("blk", ctypes.c_uint8 * 128)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.oracle_sha2_digest.argtypes = [ctypes.c_int, vp, sz, vp]
        L.oracle_sha2_digest.restype = ctypes.c_int
        L.oracle_hmac_digest.argtypes = [ctypes.c_int, vp, sz, vp, sz, vp]
        L.oracle_hmac_digest.restype = ctypes.c_int
        L.oracle_sha2_batch.argtypes = [ctypes.c_int, vp, vp, vp,
                                        ctypes.c_uint64, ctypes.c_uint32, sz,
                                        vp, ctypes.c_int]
        L.oracle_sha2_batch.restype = ctypes.c_int
        L.oracle_sha2_batch_ex.argtypes = L.oracle_sha2_batch.argtypes + [ctypes.c_int]
        L.oracle_sha2_batch_ex.restype = ctypes.c_int
        L.oracle_ph_to_iv.argtypes = [ctypes.c_uint32, ctypes.c_uint32, sz, vp]
        L.oracle_ph_to_iv.restype = ctypes.c_int
        u32, u64, i = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.oracle_hmac_batch.argtypes = [i, vp, sz, vp, vp, vp, u64, u32, sz, vp, i]
        L.oracle_ph_to_iv_batch.argtypes = [vp, vp, sz, sz, vp, i]
        L.oracle_packet_decode_batch.argtypes = [i, vp, sz, vp, sz, i, u32, u32,
                                                 i, sz, vp, vp, vp, sz, vp, vp,
                                                 vp, vp, i]
        L.oracle_packet_encode_batch.argtypes = [i, vp, sz, i, vp, vp, vp, vp, vp,
                                                 sz, vp, i]
        for f in ("oracle_hmac_batch", "oracle_ph_to_iv_batch",
                  "oracle_packet_decode_batch", "oracle_packet_encode_batch"):
            getattr(L, f).restype = ctypes.c_int
        for pfx in ("sha256", "sha384", "sha512"):
            for fn, args in (("init", [vp]), ("update", [vp, vp, sz]),
                             ("pad", [vp]), ("final", [vp, vp])):
                f = getattr(L, f"oracle_{pfx}_{fn}")
                f.argtypes = args
                f.restype = None
        _lib = L
    return _lib


def digest(alg: int, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    buf = ctypes.create_string_buffer(bytes(msg), max(len(msg), 1))
    n = lib().oracle_sha2_digest(alg, buf, len(msg), out)
    if n < 0:
        raise ValueError(f"bad alg {alg}")
    return out.raw[:n]


def hmac(alg: int, key: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    kb = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    mb = ctypes.create_string_buffer(bytes(msg), max(len(msg), 1))
    n = lib().oracle_hmac_digest(alg, kb, len(key), mb, len(msg), out)
    if n < 0:
        raise ValueError(f"bad alg {alg}")
    return out.raw[:n]


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def batch(alg: int, data: np.ndarray, offsets=None, lens=None, stride=0,
          length=0, n=None, nthreads=1, unrolled=False) -> np.ndarray:
    """CPU digests of a packet batch, same layouts as net2_sha2_batch;
    unrolled=True runs the SHA2_UNROLL_TRANSFORM form of the transforms."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = len(offsets)
    out = np.empty((n, DIGEST_LEN[alg]), dtype=np.uint8)
    rc = lib().oracle_sha2_batch_ex(alg, _ptr(data), _ptr(offsets), _ptr(lens),
                                    stride, length, n, _ptr(out), nthreads,
                                    int(unrolled))
    if rc != 0:
        raise ValueError(f"bad alg {alg}")
    return out


_ossl = None


def openssl_batch(alg: int, data: np.ndarray, offsets=None, lens=None,
                  stride=0, length=0, n=None, nthreads=1) -> np.ndarray:
    """The same batch through OpenSSL's SHA*_Init/Update/Final, the calls
    the reference's C++ layer makes (cxx_src/hash-openssl.cc:25-131); a CPU
    baseline for context (oracle/openssl_batch.c)."""
    global _ossl
    if _ossl is None:
        path = os.path.join(HERE, "libcpu_openssl.so")
        if not os.path.exists(path):
            build()
        _ossl = ctypes.CDLL(path)
        _ossl.cpu_openssl_batch.restype = ctypes.c_int
        _ossl.cpu_openssl_batch.argtypes = [
            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p,
            ctypes.c_int]
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = len(offsets)
    out = np.empty((n, DIGEST_LEN[alg]), dtype=np.uint8)
    if _ossl.cpu_openssl_batch(alg, _ptr(data), _ptr(offsets), _ptr(lens),
                               stride, length, n, _ptr(out), nthreads) != 0:
        raise ValueError(f"bad alg {alg}")
    return out


def ph_to_iv(seq: int, flags: int, ivlen: int) -> bytes:
    out = ctypes.create_string_buffer(max(ivlen, 1))
    lib().oracle_ph_to_iv(seq, flags, ivlen, out)
    return out.raw[:ivlen]


def _nthreads(nthreads):
    return nthreads if nthreads else min(16, os.cpu_count() or 1)


def _keybuf(key):
    return None if key is None else ctypes.create_string_buffer(bytes(key), max(len(key), 1))


def hmac_batch(alg: int, key: bytes, data: np.ndarray, offsets=None, lens=None,
               stride=0, length=0, n=None, nthreads=0) -> np.ndarray:
    """HMAC (alg 4..6) of every packet under one key, threaded; layouts as
    batch()."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = len(offsets)
    out = np.empty((n, DIGEST_LEN[alg]), dtype=np.uint8)
    kb = _keybuf(key)
    if lib().oracle_hmac_batch(alg, kb, len(key), _ptr(data), _ptr(offsets),
                               _ptr(lens), stride, length, n, _ptr(out),
                               _nthreads(nthreads)) != 0:
        raise ValueError(f"bad alg {alg}")
    return out


def ph_to_iv_batch(seq: np.ndarray, flags: np.ndarray, ivlen: int,
                   nthreads=0) -> np.ndarray:
    seq = np.ascontiguousarray(seq, dtype=np.uint32)
    flags = np.ascontiguousarray(flags, dtype=np.uint32)
    out = np.zeros((len(seq), max(ivlen, 1)), dtype=np.uint8)
    lib().oracle_ph_to_iv_batch(_ptr(seq), _ptr(flags), len(seq), ivlen,
                                _ptr(out), _nthreads(nthreads))
    return out[:, :ivlen]


def packet_decode_batch(hash_alg: int, key: bytes, enc_set: bool, ivlen: int,
                        data: np.ndarray, offsets, lens, alt_key=None,
                        alt_no_cutoff=False, alt_cutoff=0, rx_start=0,
                        nthreads=0):
    """The hash steps of net2_packet_decode over a burst (see
    oracle_packet_decode_batch): (result u8[n], iv u8[n, ivlen],
    seq u32[n], flags u32[n]); iv rows with no IV due are zero."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    n = len(offsets)
    res = np.full(n, 9, dtype=np.uint8)
    iv = np.zeros((n, max(ivlen, 1)), dtype=np.uint8)
    seq = np.zeros(n, dtype=np.uint32)
    fl = np.zeros(n, dtype=np.uint32)
    key = key or b""
    if lib().oracle_packet_decode_batch(
            hash_alg, _keybuf(key), len(key), _keybuf(alt_key),
            len(alt_key) if alt_key is not None else 0, int(alt_no_cutoff),
            alt_cutoff, rx_start, int(enc_set), ivlen, _ptr(data), _ptr(offsets),
            _ptr(lens), n, _ptr(res), _ptr(iv) if ivlen else None, _ptr(seq),
            _ptr(fl), _nthreads(nthreads)) != 0:
        raise ValueError(f"bad alg {hash_alg}")
    return res, iv[:, :ivlen], seq, fl


def packet_encode_batch(hash_alg: int, key: bytes, enc_set: bool, seq, flags,
                        data: np.ndarray, offsets, lens, nthreads=0):
    """The hash steps of net2_packet_encode over a burst, on a copy of data:
    (result u8[n], sealed bytes)."""
    out = np.array(data, dtype=np.uint8, copy=True)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    seq = np.ascontiguousarray(seq, dtype=np.uint32)
    flags = np.ascontiguousarray(flags, dtype=np.uint32)
    n = len(offsets)
    res = np.full(n, 9, dtype=np.uint8)
    key = key or b""
    if lib().oracle_packet_encode_batch(
            hash_alg, _keybuf(key), len(key), int(enc_set), _ptr(seq), _ptr(flags),
            _ptr(out), _ptr(offsets), _ptr(lens), n, _ptr(res),
            _nthreads(nthreads)) != 0:
        raise ValueError(f"bad alg {hash_alg}")
    return res, out
