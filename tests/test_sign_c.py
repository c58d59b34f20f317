"""The host-side C restatement of the signed-payload callers (src/sign.c,
types/signature.n2t) over the C ABI, exercised through tests/c/test_sign.c
(which restates the reference's test/sign.c)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c", "test_sign")
LIB = os.path.join(ROOT, "ilias_net2_amd", "libnet2_sign.so")
KEYS = [os.path.join(ROOT, "tests", "golden", "keys", f)
        for f in ("ecdsa_p521_priv.pem", "ecdsa_p521_pub.pem")]


def _declared(hdr):
    src = open(os.path.join(ROOT, "include", "net2", hdr)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(net2x?_\w+)\s*\(", src)) | set(
        re.findall(r"extern\s+const\s+int\s+(net2x?_\w+)\s*;", src))


def test_sign_library_exports():
    import ilias_net2_amd._lib as L
    L.lib()  # loads libnet2_sha2.so first (same process, one HIP runtime)
    lib = ctypes.CDLL(LIB)
    for name in (_declared("sign.h") | _declared("signature.h") | _declared("wire.h")
                 | _declared("signed_carver.h")):
        assert hasattr(lib, name), name
    # the reference's registry constant (include/ilias/net2/sign.h:61,
    # src/sign.c:653), as test/sign.c:66,69 pass it
    ecdsa = ctypes.c_int.in_dll(lib, "net2x_sign_ecdsa").value
    assert ecdsa == 0
    lib.net2x_sign_getname.restype = ctypes.c_char_p
    assert lib.net2x_sign_getname(ecdsa) == b"ecdsa"


def test_reference_sign_flow_cpu():
    """test/sign.c:57-185 restated: ECDSA on the host, no hashing."""
    r = subprocess.run([BIN, *KEYS, "cpu"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS cpu-only" in r.stdout


@pytest.mark.gpu
def test_sign_and_signatures_gpu():
    """Fingerprint, signature create/validate single and batched: every
    digest from the GPU path, cross-checked by verifying with an
    OpenSSL-computed digest."""
    r = subprocess.run([BIN, *KEYS], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS (0 failures)" in r.stdout


# ---- the hash-only tick (net2_sc_hash_req), VERDICT round 3 item 1 --------

class HashReq(ctypes.Structure):
    pass


HASH_CB = ctypes.CFUNCTYPE(None, ctypes.POINTER(HashReq), ctypes.c_void_p)
HashReq._fields_ = [("payload", ctypes.c_void_p), ("iovcnt", ctypes.c_size_t),
                    ("hash_alg", ctypes.c_int), ("done", HASH_CB),
                    ("arg", ctypes.c_void_p), ("rc", ctypes.c_int),
                    ("digestlen", ctypes.c_uint32),
                    ("digest", ctypes.c_uint8 * 64)]


def test_hash_req_layout():
    """The ctypes mirror matches include/net2/signed_carver.h (LP64)."""
    assert ctypes.sizeof(HashReq) == 112
    assert HashReq.rc.offset == 40 and HashReq.digest.offset == 48


@pytest.mark.gpu
def test_hash_tick_4096_x_1k_against_oracle(oracle_mod):
    """net2_sc_hash_tick at BASELINE configs[0]'s shape, 4096 x 1 KiB:
    SHA-256 / 384 / 512 mixed, every 7th payload split over two iovecs,
    one keyed row (EINVAL); every digest against the oracle, every callback
    exactly once, with its own request."""
    import numpy as np
    import ilias_net2_amd._lib as L
    from synth import random_bytes
    L.lib()
    lib = ctypes.CDLL(LIB)
    lib.net2_sc_hash_tick.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    lib.net2_sc_hash_tick.restype = ctypes.c_int
    N, LEN = 4096, 1024
    data = random_bytes(41, N * LEN)
    base = data.ctypes.data
    iov = (L.IOVec * (2 * N))()
    reqs = (HashReq * N)()
    calls = np.zeros(N, dtype=np.int64)
    addr0 = ctypes.addressof(reqs)
    wrong = []  # an assert inside a ctypes callback would not reach pytest

    def done(req, arg):
        i = (ctypes.addressof(req.contents) - addr0) // ctypes.sizeof(HashReq)
        if arg != i + 1:
            wrong.append(i)
        calls[i] += 1
    cb = HASH_CB(done)
    for i in range(N):
        split = i % 7 == 0
        iov[2 * i].iov_base = base + i * LEN
        iov[2 * i].iov_len = 333 if split else LEN
        iov[2 * i + 1].iov_base = base + i * LEN + 333
        iov[2 * i + 1].iov_len = LEN - 333
        reqs[i].payload = ctypes.addressof(iov) + 2 * i * ctypes.sizeof(L.IOVec)
        reqs[i].iovcnt = 2 if split else 1
        reqs[i].hash_alg = 1 + i % 3
        reqs[i].done = cb
        reqs[i].arg = i + 1
    reqs[N - 1].hash_alg = 6  # HMAC-SHA512: keyed, not a sighash
    assert lib.net2_sc_hash_tick(reqs, N, 8) == 0
    assert (calls == 1).all() and not wrong
    assert reqs[N - 1].rc == 22 and reqs[N - 1].digestlen == 0  # EINVAL
    for alg in (1, 2, 3):
        idx = [i for i in range(N - 1) if 1 + i % 3 == alg]
        want = oracle_mod.batch(alg, data, stride=LEN, length=LEN, n=N)
        hl = oracle_mod.DIGEST_LEN[alg]
        for i in idx:
            assert reqs[i].rc == 0 and reqs[i].digestlen == hl, i
            assert bytes(reqs[i].digest[:hl]) == want[i].tobytes(), i


@pytest.mark.gpu
def test_hash_tick_few_long_payloads(oracle_mod):
    """A tick of a few long payloads (the reference's maximum, 65,536 B,
    src/carver.c:150,161, and above) takes the coalescer's wave-per-message
    form (one request per payload, submitted at once); digests against the
    oracle, multi-segment payloads included."""
    import numpy as np
    import ilias_net2_amd._lib as L
    from synth import random_bytes
    L.lib()
    lib = ctypes.CDLL(LIB)
    lib.net2_sc_hash_tick.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    sizes = [65536, 70001, 65536, 100000, 9000]
    datas = [random_bytes(50 + i, n) for i, n in enumerate(sizes)]
    iov = (L.IOVec * (2 * len(sizes)))()
    reqs = (HashReq * len(sizes))()
    for i, d in enumerate(datas):
        cut = 1000 if i % 2 else len(d)
        iov[2 * i].iov_base = d.ctypes.data
        iov[2 * i].iov_len = cut
        iov[2 * i + 1].iov_base = d.ctypes.data + cut
        iov[2 * i + 1].iov_len = len(d) - cut
        reqs[i].payload = ctypes.addressof(iov) + 2 * i * ctypes.sizeof(L.IOVec)
        reqs[i].iovcnt = 2
        reqs[i].hash_alg = (1, 3, 2, 3, 1)[i]
    assert lib.net2_sc_hash_tick(reqs, len(sizes), 4) == 0
    for i, d in enumerate(datas):
        alg = reqs[i].hash_alg
        want = oracle_mod.digest(alg, d.tobytes())
        assert reqs[i].rc == 0 and reqs[i].digestlen == len(want), i
        assert bytes(reqs[i].digest[:len(want)]) == want, i
