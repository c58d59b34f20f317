"""The single-message entry points on the GPU: the streaming SHA2_CTX
interface of src/sha2.c (include/net2/sha2.h), net2_hashctx_hashiov and
net2_ph_to_iv, all running through the request coalescer
(ilias_net2_amd/csrc/sha2_coalesce.cpp), alone and from many threads at once.

The streaming calls are compared with the oracle's restatement of the same
calls (oracle/sha2_oracle.c) context byte for context byte after every call:
state, bit count and the buffer as src/sha2.c leaves it
(src/sha2.c:449-563, :738-919).
"""
import ctypes
import errno
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

PFX = {1: "SHA256", 2: "SHA384", 3: "SHA512"}
OPFX = {1: "sha256", 2: "sha384", 3: "sha512"}
DL = {1: 32, 2: 48, 3: 64}
BL = {1: 64, 2: 128, 3: 128}


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (HIP device not visible)")
    from ilias_net2_amd import _lib
    assert _lib.device_count() >= 1
    return _lib.lib()


def _ctx():
    return ctypes.create_string_buffer(208)


def _buf(b: bytes):
    return ctypes.create_string_buffer(b, max(len(b), 1))


def test_streaming_matches_oracle_call_by_call(L, oracle_mod):
    O = oracle_mod.lib()
    rng = np.random.default_rng(1)
    for alg in (1, 2, 3):
        p, op = PFX[alg], OPFX[alg]
        for n in (0, 1, 55, 56, 63, 64, 65, 111, 112, 119, 120, 127, 128,
                  129, 1000, 4097):
            m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            cuts = sorted(rng.integers(0, n + 1, 5).tolist())
            chunks = [m[a:b] for a, b in zip([0] + cuts, cuts + [n])]
            c, oc = _ctx(), _ctx()
            getattr(L, p + "Init")(c)
            getattr(O, f"oracle_{op}_init")(oc)
            assert c.raw == oc.raw
            for ch in chunks:
                b = _buf(ch)
                getattr(L, p + "Update")(c, b, len(ch))
                getattr(O, f"oracle_{op}_update")(oc, b, len(ch))
                assert c.raw == oc.raw, (alg, n, len(ch))
            d, od = ctypes.create_string_buffer(64), ctypes.create_string_buffer(64)
            getattr(L, p + "Final")(d, c)
            getattr(O, f"oracle_{op}_final")(od, oc)
            assert d.raw[:DL[alg]] == od.raw[:DL[alg]] == oracle_mod.digest(alg, m)
            assert c.raw == oc.raw == b"\0" * 208


def test_long_update_in_chunks(L, oracle_mod, monkeypatch):
    """An Update longer than the per-request chunk goes through in several
    coalesced requests chained through a local state (small chunks forced
    with NET2_SHA2_STREAM_CHUNK): the context matches the oracle's after
    every call, whatever the chunk and the buffered head."""
    O = oracle_mod.lib()
    rng = np.random.default_rng(3)
    for chunk in ("64", "4096", "65600"):
        monkeypatch.setenv("NET2_SHA2_STREAM_CHUNK", chunk)
        for alg in (1, 2, 3):
            p, op = PFX[alg], OPFX[alg]
            m = rng.integers(0, 256, 300001, dtype=np.uint8).tobytes()
            c, oc = _ctx(), _ctx()
            getattr(L, p + "Init")(c)
            getattr(O, f"oracle_{op}_init")(oc)
            for ch in (m[:13], m[13:250013], m[250013:]):
                b = _buf(ch)
                getattr(L, p + "Update")(c, b, len(ch))
                getattr(O, f"oracle_{op}_update")(oc, b, len(ch))
                assert c.raw == oc.raw, (chunk, alg, len(ch))
            d = ctypes.create_string_buffer(64)
            getattr(L, p + "Final")(d, c)
            assert d.raw[:DL[alg]] == oracle_mod.digest(alg, m), (chunk, alg)


def test_pad_and_final_null(L, oracle_mod):
    """Pad alone, and Final(NULL) keeping the padded context for SHA-256 /
    SHA-512 while SHA-384 zeroes it (src/sha2.c:551-562, :918)."""
    O = oracle_mod.lib()
    for alg in (1, 2, 3):
        p, op = PFX[alg], OPFX[alg]
        for n in (3, BL[alg] - 9, BL[alg] - 8, BL[alg]):
            m = _buf(bytes(range(n)))
            c, oc = _ctx(), _ctx()
            getattr(L, p + "Init")(c)
            getattr(O, f"oracle_{op}_init")(oc)
            getattr(L, p + "Update")(c, m, n)
            getattr(O, f"oracle_{op}_update")(oc, m, n)
            getattr(L, p + "Pad")(c)
            getattr(O, f"oracle_{op}_pad")(oc)
            assert c.raw == oc.raw, (alg, n)
            getattr(L, p + "Final")(None, c)
            getattr(O, f"oracle_{op}_final")(None, oc)
            assert c.raw == oc.raw, (alg, n)
            assert (c.raw == b"\0" * 208) == (alg == 2)


def test_transform(L, oracle_mod):
    O = oracle_mod.lib()
    rng = np.random.default_rng(2)
    for alg, words, ct in ((1, 8, ctypes.c_uint32), (2, 8, ctypes.c_uint64),
                           (3, 8, ctypes.c_uint64)):
        blk = _buf(rng.integers(0, 256, BL[alg], dtype=np.uint8).tobytes())
        st = (ct * words)(*[int(x) for x in rng.integers(0, 2**31, words)])
        ost = (ct * words)(*st)
        getattr(L, PFX[alg] + "Transform")(st, blk)
        getattr(O, "oracle_sha256_transform" if alg == 1 else
                "oracle_sha512_transform")(ost, blk)
        assert list(st) == list(ost)
        # error form: same result, state unchanged on a bad row
        st2 = (ct * words)(*[int(x) for x in range(words)])
        ost2 = (ct * words)(*st2)
        assert L.net2_sha2_ctx_transform(alg, st2, blk) == 0
        getattr(O, "oracle_sha256_transform" if alg == 1 else
                "oracle_sha512_transform")(ost2, blk)
        assert list(st2) == list(ost2)


def test_hashiov_sizes(L, oracle_mod):
    """Empty, boundary and multi-MiB messages (the staging grows), every row."""
    from ilias_net2_amd import hash as h
    rng = np.random.default_rng(3)
    for n in (0, 1, 55, 56, 64, 111, 112, 128, 1500, 65536, 5 << 20):
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for alg in (1, 2, 3):
            assert h.hashbuf(alg, b"", m) == oracle_mod.digest(alg, m), (alg, n)
        for alg in (4, 5, 6):
            key = bytes(range(DL[alg - 3]))
            assert h.hashbuf(alg, key, m) == oracle_mod.hmac(alg, key, m), (alg, n)


def test_hashiov_long_messages_streamed(L, oracle_mod, monkeypatch):
    """A message longer than NET2_SHA2_STREAM_CHUNK (64 MiB by default; 4 KiB
    here) goes through the streaming context in chunks instead of one
    request, keyed rows as RFC 2104 over it: every row, segments of odd
    sizes, against the oracle; the threshold itself takes the one-request
    path."""
    import ctypes as ct
    monkeypatch.setenv("NET2_SHA2_STREAM_CHUNK", "4096")
    rng = np.random.default_rng(5)
    for n in (4096, 4097, 100003):
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        cuts = sorted(rng.integers(0, n + 1, 4).tolist())
        segs = [m[a:b] for a, b in zip([0] + cuts, cuts + [n])]
        bufs = [ct.create_string_buffer(x, max(len(x), 1)) for x in segs]

        from ilias_net2_amd._lib import IOVec
        iov = (IOVec * len(segs))(*[IOVec(ct.cast(b, ct.c_void_p), len(x))
                                    for b, x in zip(bufs, segs)])
        for alg in range(1, 7):
            dl = DL[alg if alg <= 3 else alg - 3]
            key = bytes(range(dl)) if alg > 3 else b""
            kb = ct.create_string_buffer(key, max(len(key), 1))
            out = ct.create_string_buffer(64)
            assert L.net2_hashctx_hashiov(alg, kb if key else None, len(key), iov,
                                          len(segs), out, 64) == 0
            want = oracle_mod.digest(alg, m) if alg <= 3 else \
                oracle_mod.hmac(alg, key, m)
            assert out.raw[:dl] == want, (alg, n)


def test_hashiov_streamed_gathers_small_segments(L, oracle_mod, monkeypatch):
    """A long message made of many small iovecs goes to the GPU in requests
    of about one stream chunk, not one per segment: 1,000
    segments of 1-300 bytes with a 4 KiB chunk take ~40 launches, and the
    digest / HMAC equal the oracle's."""
    import ctypes as ct
    from ilias_net2_amd._lib import IOVec
    monkeypatch.setenv("NET2_SHA2_STREAM_CHUNK", "4096")
    rng = np.random.default_rng(11)
    sizes = rng.integers(1, 301, 1000)
    m = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8).tobytes()
    cuts = np.concatenate([[0], np.cumsum(sizes)])
    bufs = [ct.create_string_buffer(m[a:b], b - a) for a, b in zip(cuts, cuts[1:])]
    iov = (IOVec * len(bufs))(*[IOVec(ct.cast(b, ct.c_void_p), len(b)) for b in bufs])
    for alg in (1, 3, 6):
        key = bytes(range(64)) if alg == 6 else b""
        kb = ct.create_string_buffer(key, max(len(key), 1))
        out = ct.create_string_buffer(64)
        c0, n0 = _stats(L)
        assert L.net2_hashctx_hashiov(alg, kb if key else None, len(key), iov,
                                      len(bufs), out, 64) == 0
        c1, n1 = _stats(L)
        want = oracle_mod.digest(alg, m) if alg <= 3 else oracle_mod.hmac(alg, key, m)
        assert out.raw[:len(want)] == want, alg
        assert n1 - n0 <= len(m) // 4096 + 8, (alg, n1 - n0)


def test_long_job_in_a_batch_of_small_ones(L, oracle_mod):
    """A long request (1,024 blocks or more) in a batch of many small ones
    takes a wave of its own in a separate launch while the small ones keep
    the lane form: 32 threads of 1 KiB calls and 2 threads
    of 200 KiB calls at once, every digest against the oracle."""
    import ctypes as ct
    from ilias_net2_amd._lib import IOVec
    rng = np.random.default_rng(12)
    small = [rng.integers(0, 256, 1024, dtype=np.uint8).tobytes() for _ in range(32)]
    big = [rng.integers(0, 256, 200 * 1024 + 17, dtype=np.uint8).tobytes()
           for _ in range(2)]
    bad = []

    def run(msg, alg, reps):
        b = ct.create_string_buffer(msg, len(msg))
        iov = (IOVec * 1)(IOVec(ct.cast(b, ct.c_void_p), len(msg)))
        want = oracle_mod.digest(alg, msg)
        for _ in range(reps):
            out = ct.create_string_buffer(64)
            if L.net2_hashctx_hashiov(alg, None, 0, iov, 1, out, 64) != 0 or \
                    out.raw[:len(want)] != want:
                bad.append((alg, len(msg)))
    ths = [threading.Thread(target=run, args=(m, 1 + 2 * (i % 2), 40))
           for i, m in enumerate(small)]
    ths += [threading.Thread(target=run, args=(m, 1 + 2 * i, 6))
            for i, m in enumerate(big)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not bad, bad[:4]


def _registry_key(key: bytes, alg: int) -> bytes:
    """RFC 2104: K' is K (hashed first if longer than the block) zero-padded
    to the block, so any zero extension of that up to the block gives the
    same MAC -- here to the registry's key length (= hashlen,
    hash-openssl.cc:417-429)."""
    import hashlib
    h = {4: hashlib.sha256, 5: hashlib.sha384, 6: hashlib.sha512}[alg]
    blk = 64 if alg == 4 else 128
    k = h(key).digest() if len(key) > blk else key
    kl = {4: 32, 5: 48, 6: 64}[alg]
    assert len(k) <= kl
    return k + b"\0" * (kl - len(k))


def test_rfc4231_on_gpu(L, golden):
    """RFC 4231 cases 1-7 through the keyed rows of net2_hashctx_hashiov,
    every key expressed at the registry's key length."""
    from ilias_net2_amd import hash as h
    for c in golden["kat"]["rfc4231"]:
        key, data = bytes.fromhex(c["key"]), bytes.fromhex(c["data"])
        for alg, name in ((4, "HMAC-SHA256"), (5, "HMAC-SHA384"),
                          (6, "HMAC-SHA512")):
            want = c[name]
            got = h.hashbuf(alg, _registry_key(key, alg), data).hex()
            assert got[:len(want)] == want, (c["case"], name)


def test_many_threads_mixed(L, oracle_mod):
    """64 threads at once, mixing digests, HMACs, streaming contexts and
    IV derivations of every row, so batches hold SHA-256 and SHA-512 jobs
    of all kinds; every result against the oracle."""
    from ilias_net2_amd import hash as h

    class PH(ctypes.Structure):
        _fields_ = [("seq", ctypes.c_uint32), ("flags", ctypes.c_uint32)]
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(100 + t)
            for j in range(30):
                kind = (t + j) % 4
                n = int(rng.integers(0, 2500))
                m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
                alg = 1 + int(rng.integers(0, 3))
                if kind == 0:
                    if h.hashbuf(alg, b"", m) != oracle_mod.digest(alg, m):
                        errors.append(("digest", t, j))
                elif kind == 1:
                    key = rng.integers(0, 256, DL[alg], dtype=np.uint8).tobytes()
                    if h.hashbuf(alg + 3, key, m) != oracle_mod.hmac(alg + 3, key, m):
                        errors.append(("hmac", t, j))
                elif kind == 2:
                    c = _ctx()
                    getattr(L, PFX[alg] + "Init")(c)
                    for a in range(0, n, 333):
                        b = _buf(m[a:a + 333])
                        getattr(L, PFX[alg] + "Update")(c, b, len(m[a:a + 333]))
                    d = ctypes.create_string_buffer(64)
                    getattr(L, PFX[alg] + "Final")(d, c)
                    if d.raw[:DL[alg]] != oracle_mod.digest(alg, m):
                        errors.append(("ctx", t, j))
                else:
                    seq, fl = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
                    ivlen = int(rng.integers(1, 80))
                    out = ctypes.create_string_buffer(ivlen)
                    rc = L.net2_ph_to_iv_buf(ctypes.byref(PH(seq, fl)), ivlen, out)
                    if rc != 0 or out.raw[:ivlen] != oracle_mod.ph_to_iv(seq, fl, ivlen):
                        errors.append(("iv", t, j, rc))
        except Exception as e:  # noqa: BLE001
            errors.append(("exc", t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(64)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:5]


def _stats(L):
    c, n = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.net2_coalesce_stats(-1, ctypes.byref(c), ctypes.byref(n)) == 0
    return c.value, n.value


def test_coalesced_batches_form(L, oracle_mod):
    """Under concurrency the calls really share launches: 32 threads x 50
    calls of a 1 KiB SHA-512 straight through net2_hashctx_hashiov (ctypes
    drops the GIL for the call, so the calls overlap in the library) take
    far fewer launches than calls (net2_coalesce_stats), and every digest is
    right.  tools/coalesce_bench.c measures the rates."""
    from ilias_net2_amd import _lib
    m = bytes(range(256)) * 4
    want = oracle_mod.digest(3, m)
    buf = ctypes.create_string_buffer(m, len(m))
    iov = (_lib.IOVec * 1)()
    iov[0].iov_base = ctypes.cast(buf, ctypes.c_void_p)
    iov[0].iov_len = len(m)

    def one():
        out = ctypes.create_string_buffer(64)
        assert L.net2_hashctx_hashiov(3, None, 0, iov, 1, out, 64) == 0
        return out.raw
    assert one() == want
    c0, n0 = _stats(L)
    for _ in range(20):              # one at a time: a launch per call
        one()
    c1, n1 = _stats(L)
    assert (c1 - c0, n1 - n0) == (20, 20)
    bad = []

    def worker():
        for _ in range(50):
            if one() != want:
                bad.append(1)
    ths = [threading.Thread(target=worker) for _ in range(32)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    c2, n2 = _stats(L)
    assert not bad
    assert c2 - c1 == 1600
    # 1,600 calls from 32 threads: batches of several calls each
    assert n2 - n1 < 1600 / 2, (c2 - c1, n2 - n1)
    # the stats of a device index out of range
    assert L.net2_coalesce_stats(99, None, None) == errno.EINVAL


_FORM_CHECK = r'''
import sys, ctypes
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np
import torch  # noqa: F401  (one HIP runtime: torch first)
from ilias_net2_amd import hash as h, _lib
from oracle import oracle
L = _lib.lib()
rng = np.random.default_rng(9)
bad = 0
for n in (0, 1, 63, 64, 119, 128, 1024, 5000, 70000):
    m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    for alg in (1, 2, 3):
        bad += h.hashbuf(alg, b"", m) != oracle.digest(alg, m)
        key = bytes(range(7, 7 + {1: 32, 2: 48, 3: 64}[alg]))
        bad += h.hashbuf(alg + 3, key, m) != oracle.hmac(alg + 3, key, m)
        ctx = ctypes.create_string_buffer(208)
        L.net2_sha2_ctx_init(alg, ctx)
        for a in range(0, n, 999):
            seg = m[a:a + 999]
            L.net2_sha2_ctx_update(alg, ctx, seg, len(seg))
        d = ctypes.create_string_buffer(64)
        L.net2_sha2_ctx_final(alg, d, ctx)
        bad += d.raw[:{1: 32, 2: 48, 3: 64}[alg]] != oracle.digest(alg, m)
print("BAD", bad)
'''


@pytest.mark.parametrize("mode", ["1", "2", "2-chunked"])
def test_wave_and_lane_job_forms(L, mode):
    """Both kernels behind the coalescer -- one wave per job (the latency
    form, chosen automatically for batches of up to 16 jobs,
    kWaveJobsMax in csrc/sha2_coalesce.cpp, or when a job has 1,024 blocks
    or more, kWaveBlocks) and one lane per job -- forced in a fresh process
    each (NET2_COALESCE_JOBMODE), messages up to 70,000 bytes (more than 64
    blocks: the wave form's chunk loop; with 4,096-byte lane-form pieces,
    the lane form's)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NET2_COALESCE_JOBMODE=mode[0])
    if mode.endswith("chunked"):
        # the lane form absorbs a job in < 4 GiB pieces (a
        # 4 GiB job was truncated); 4,096-byte pieces run that split on
        # these messages (a 4 GiB one would take a lane minutes)
        env["NET2_COALESCE_JOB_CHUNK"] = "32"
    r = subprocess.run([sys.executable, "-c", _FORM_CHECK], cwd=root, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "BAD 0" in r.stdout, r.stdout + r.stderr
