"""Packet bursts from host memory (net2_packet_decode_burst_host /
net2_packet_encode_burst_host): the hash steps of net2_packet_decode /
_encode (types/packet.n2t:170-336 / :341-463) for datagrams that live in host
memory, as the reference's do -- received one at a time by
net2_sockdgram_recv (src/sockdgram.c:67-108) and decoded at
src/connection.c:199; built by gather() (src/connection.c:336-339) and
encoded at :467.

Every result is compared with the oracle's restatement of those functions
(oracle_packet_decode_batch / _encode_batch, pinned in
tests/test_oracle_batch.py): codes, sealed bytes, decoded headers and IVs,
intact and tampered, from pageable and from page-locked memory, on one device
and sliced over several (NET2_SHA2_VIRTUAL_DEVICES lists the box's GPU k
times, so every slice runs its own thread, staging and streams).
"""
import ctypes
import errno
import os

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

PH_ENCRYPTED, PH_SIGNED, PH_ALTKEY = 0x1, 0x2, 0x80000000
OK, RESOURCE, BAD, UNSAFE = 0, 1, 2, 3
HL = {0: 0, 4: 32, 5: 48, 6: 64}
CPU_THREADS = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (HIP device not visible)")
    from ilias_net2_amd import _lib
    assert _lib.device_count() >= 1
    return torch.device("cuda:0")


@pytest.fixture
def virtual(monkeypatch):
    def set_k(k):
        monkeypatch.setenv("NET2_SHA2_VIRTUAL_DEVICES", str(k))
        monkeypatch.setenv("NET2_SHA2_SLICE_MIN_BYTES", "0")
    yield set_k


def _p(a):
    return a.ctypes.data if a is not None else None


def pinned(shape, dtype):
    """A page-locked host array (torch pin_memory), as a numpy view."""
    t = torch.empty(shape, dtype={np.uint8: torch.uint8, np.uint32: torch.int32,
                                  np.uint64: torch.int64}[dtype], pin_memory=True)
    return t.numpy().view(dtype)


def encode_host(L, hash_alg, key, enc_set, seq, flags, data, offs, lens,
                max_devices=0, result=None):
    res = np.full(len(offs), 9, dtype=np.uint8) if result is None else result
    rc = L.net2_packet_encode_burst_host(
        hash_alg, key or None, len(key), int(enc_set), _p(seq), _p(flags),
        _p(data), _p(offs), _p(lens), len(offs), _p(res), max_devices)
    assert rc == 0, rc
    return res


def decode_host(L, keys, ivlen, data, offs, lens, max_devices=0, out=None):
    n = len(offs)
    if out is None:
        out = dict(res=np.full(n, 9, dtype=np.uint8),
                   iv=np.zeros((n, max(ivlen, 1)), dtype=np.uint8),
                   seq=np.zeros(n, dtype=np.uint32),
                   fl=np.zeros(n, dtype=np.uint32))
    rc = L.net2_packet_decode_burst_host(
        ctypes.byref(keys), ivlen, _p(data), _p(offs), _p(lens), n,
        _p(out["res"]), _p(out["iv"]) if ivlen else None, _p(out["seq"]),
        _p(out["fl"]), max_devices)
    assert rc == 0, rc
    return out


def rx_keys(hash_alg, key, enc_set, alt=None, no_cutoff=0, cutoff=0, rx_start=0):
    from ilias_net2_amd import _lib
    kb = ctypes.create_string_buffer(key, max(len(key), 1))
    ab = ctypes.create_string_buffer(alt, len(alt)) if alt else None
    ks = _lib.BurstRxKeys(hash_alg, ctypes.cast(kb, ctypes.c_void_p) if key else None,
                          len(key), int(enc_set),
                          ctypes.cast(ab, ctypes.c_void_p) if alt else None,
                          len(alt) if alt else 0, no_cutoff, cutoff, rx_start)
    ks._keep = (kb, ab)
    return ks


def check_decode(got, want, ivlen):
    o_res, o_iv, o_seq, o_fl = want
    assert np.array_equal(got["res"], o_res), np.nonzero(got["res"] != o_res)[0][:8]
    # headers are decoded for every datagram of at least 8 bytes; the
    # oracle leaves the others zero, as the kernels do
    assert np.array_equal(got["seq"], o_seq)
    assert np.array_equal(got["fl"], o_fl)
    if ivlen:
        ok = o_res == OK
        assert np.array_equal(got["iv"][ok, :ivlen], o_iv[ok])


SETUPS = [(6, True, 16), (4, True, 16), (5, False, 0), (0, True, 32),
          (0, False, 0), (6, True, 64)]


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("hash_alg,enc_set,ivlen", SETUPS)
def test_host_bursts_against_oracle(dev, virtual, oracle_mod, k, hash_alg,
                                    enc_set, ivlen):
    """Mixed flags (wrong, extra, PH_ALTKEY bits), slots without room, runts
    and tampered bytes under every key set-up, byte-aligned datagrams with
    gaps between them; TX then RX, each against the oracle, sliced over k
    devices."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    virtual(k)
    rng = np.random.default_rng(3000 + 10 * hash_alg + ivlen + enc_set + 100 * k)
    n = 20011
    key = rng.integers(0, 256, HL[hash_alg], dtype=np.uint8).tobytes()
    want_flags = (PH_SIGNED if hash_alg else 0) | (PH_ENCRYPTED if enc_set else 0)
    flags = np.full(n, want_flags, dtype=np.uint32)
    pick = rng.random(n)
    flags[pick < 0.1] ^= PH_SIGNED
    flags[(pick >= 0.1) & (pick < 0.2)] ^= PH_ENCRYPTED
    flags[(pick >= 0.2) & (pick < 0.3)] |= PH_ALTKEY | 0x10
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    plen = rng.choice([0, 1, 17, 64, 500, 1472], n)
    hl = np.where(flags & PH_SIGNED, HL[hash_alg], 0)
    slot = (8 + hl + plen).astype(np.uint32)
    short = rng.random(n) < 0.03
    slot[short] = rng.integers(0, 8 + HL[hash_alg] + 1, short.sum())
    data, offs = synth.packed(3100 + hash_alg, slot, align=1, gap=3)
    offs = offs.astype(np.uint64)

    # ---- TX ------------------------------------------------------------
    o_res, o_sealed = oracle_mod.packet_encode_batch(
        hash_alg, key, enc_set, seq, flags, data, offs, slot, nthreads=CPU_THREADS)
    tx = data.copy()
    res = encode_host(L, hash_alg, key, enc_set, seq, flags, tx, offs, slot)
    assert np.array_equal(res, o_res)
    assert np.array_equal(tx, o_sealed)          # every byte, gaps included

    # ---- RX: what TX sealed, plus tampered bytes and runts ----------------
    rx = tx.copy()
    lens = slot.copy()
    tamper = rng.random(n)
    for i in np.nonzero((tamper < 0.05) & (lens > 8))[0]:
        rx[int(offs[i]) + 8 + int(rng.integers(0, lens[i] - 8))] ^= 0x40
    runt = (tamper >= 0.05) & (tamper < 0.08)
    lens[runt] = rng.integers(0, 8, runt.sum())
    want = oracle_mod.packet_decode_batch(hash_alg, key, enc_set, ivlen, rx, offs,
                                          lens, nthreads=CPU_THREADS)
    got = decode_host(L, rx_keys(hash_alg, key, enc_set), ivlen, rx, offs, lens)
    check_decode(got, want, ivlen)
    assert (want[0] == OK).sum() > n // 2 and (want[0] == BAD).sum() > 0
    # no header outputs asked for: the codes and IVs alone
    out = dict(res=np.full(n, 9, dtype=np.uint8),
               iv=np.zeros((n, max(ivlen, 1)), dtype=np.uint8), seq=None, fl=None)
    rc = L.net2_packet_decode_burst_host(
        ctypes.byref(rx_keys(hash_alg, key, enc_set)), ivlen, _p(rx), _p(offs),
        _p(lens), n, _p(out["res"]), _p(out["iv"]) if ivlen else None, None, None, 0)
    assert rc == 0
    assert np.array_equal(out["res"], want[0])


def test_host_burst_alternate_key(dev, oracle_mod):
    """A burst received during a key rollover (net2_ck_rx_key,
    src/conn_keys.c:447-476), the window start wrapping: the alternate key's
    midstates reach the kernel from the host too."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(71)
    n, hash_alg, ivlen = 30000, 6, 16
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    alt = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    rx_start = 0xfffff000
    cutoff = (rx_start + 12000) & 0xffffffff
    seq = ((rx_start + rng.integers(0, 30000, n)) & 0xffffffff).astype(np.uint32)
    flags = np.full(n, PH_SIGNED | PH_ENCRYPTED, dtype=np.uint32)
    flags[rng.random(n) < 0.3] |= PH_ALTKEY
    plen = rng.choice([0, 5, 64, 300, 1400], n).astype(np.uint32)
    lens = 8 + 64 + plen
    data, offs = synth.packed(72, lens, align=1)
    offs = offs.astype(np.uint64)
    # seal half with the active key, half with the alternate one
    half = rng.random(n) < 0.5
    for sel, k in ((half, key), (~half, alt)):
        idx = np.nonzero(sel)[0]
        r, sealed = oracle_mod.packet_encode_batch(
            hash_alg, k, True, seq[idx], flags[idx], data, offs[idx], lens[idx],
            nthreads=CPU_THREADS)
        assert (r == OK).all()
        for i in idx:
            a = int(offs[i])
            data[a:a + 72] = sealed[a:a + 72]
    want = oracle_mod.packet_decode_batch(
        hash_alg, key, True, ivlen, data, offs, lens, alt_key=alt,
        alt_no_cutoff=False, alt_cutoff=cutoff, rx_start=rx_start,
        nthreads=CPU_THREADS)
    assert 0 < (want[0] == OK).sum() < n
    got = decode_host(L, rx_keys(hash_alg, key, True, alt, 0, cutoff, rx_start),
                      ivlen, data, offs, lens)
    check_decode(got, want, ivlen)


def _mtu_burst(n, seed):
    rng = np.random.default_rng(seed)
    lens = rng.choice(np.array([136, 584, 1500], dtype=np.uint32), n)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    flags = np.full(n, PH_SIGNED | PH_ENCRYPTED, dtype=np.uint32)
    return data, offs, lens, seq, flags


@pytest.mark.parametrize("memory", ["pageable", "pinned"])
def test_host_burst_full_size(dev, oracle_mod, memory):
    """The burst bench shape end to end at full size: 1 M wire datagrams of
    {136, 584, 1500} B in host memory (HMAC-SHA512, 16-byte IVs).  TX seals
    every slot -- every byte of the buffer against the oracle -- then RX
    decodes them intact and with 4,096 chosen datagrams tampered: every code,
    header and IV against the oracle."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    n, alg, ivlen = 1 << 20, 6, 16
    data, offs, lens, seq, flags = _mtu_burst(n, 43)
    key = bytes(range(11, 75))
    o_res, o_sealed = oracle_mod.packet_encode_batch(
        alg, key, True, seq, flags, data, offs, lens, nthreads=CPU_THREADS)
    assert (o_res == OK).all()
    if memory == "pinned":
        buf = pinned(data.shape, np.uint8)
        buf[:] = data
        res = pinned((n,), np.uint8)
        out = dict(res=pinned((n,), np.uint8), iv=pinned((n, ivlen), np.uint8),
                   seq=pinned((n,), np.uint32), fl=pinned((n,), np.uint32))
    else:
        buf = data.copy()
        res = np.full(n, 9, dtype=np.uint8)
        out = None
    encode_host(L, alg, key, True, seq, flags, buf, offs, lens, result=res)
    assert np.array_equal(res, o_res)
    assert np.array_equal(buf, o_sealed)
    del o_sealed
    got = decode_host(L, rx_keys(alg, key, True), ivlen, buf, offs, lens, out=out)
    want = oracle_mod.packet_decode_batch(alg, key, True, ivlen, buf, offs, lens,
                                          nthreads=CPU_THREADS)
    check_decode(got, want, ivlen)
    assert (got["res"] == OK).all()
    assert np.array_equal(got["seq"], seq) and np.array_equal(got["fl"], flags)
    rng = np.random.default_rng(44)
    bad = np.sort(rng.choice(n, 4096, replace=False))
    pos = offs[bad] + 8 + rng.integers(0, lens[bad] - 8).astype(np.uint64)
    buf[pos.astype(np.int64)] ^= 0x20
    got = decode_host(L, rx_keys(alg, key, True), ivlen, buf, offs, lens, out=out)
    want = oracle_mod.packet_decode_batch(alg, key, True, ivlen, buf, offs, lens,
                                          nthreads=CPU_THREADS)
    check_decode(got, want, ivlen)
    assert np.array_equal(np.nonzero(got["res"])[0], bad)


def test_host_burst_mixed_memory_and_devices(dev, virtual, oracle_mod):
    """Results split between page-locked and pageable arrays (each output
    chooses its own path), the burst sliced over 3 devices, repeated so the
    slots' staging is reused with other chunk sizes."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    virtual(3)
    n, alg, ivlen = 150001, 4, 16
    data, offs, lens, seq, flags = _mtu_burst(n, 45)
    key = bytes(range(32))
    buf = data.copy()
    res = pinned((n,), np.uint8)
    encode_host(L, alg, key, True, seq, flags, buf, offs, lens, result=res)
    assert (res == OK).all()
    for rep, m in enumerate((n, n // 2 + 1, 1000, n)):
        o = offs[:m]
        out = dict(res=np.full(m, 9, dtype=np.uint8), iv=pinned((m, ivlen), np.uint8),
                   seq=np.zeros(m, dtype=np.uint32), fl=pinned((m,), np.uint32))
        got = decode_host(L, rx_keys(alg, key, True), ivlen, buf, o, lens[:m],
                          max_devices=3, out=out)
        want = oracle_mod.packet_decode_batch(alg, key, True, ivlen, buf, o, lens[:m],
                                              nthreads=CPU_THREADS)
        check_decode(got, want, ivlen)
        assert (got["res"] == OK).all(), rep


def test_host_burst_argument_errors(dev):
    from ilias_net2_amd import _lib
    L = _lib.lib()
    d = np.zeros(256, dtype=np.uint8)
    o = np.zeros(4, dtype=np.uint64)
    ln = np.full(4, 8, dtype=np.uint32)
    r = np.zeros(4, dtype=np.uint8)
    s = np.zeros(4, dtype=np.uint32)
    k = rx_keys(4, b"k" * 31, True)      # wrong key length
    assert L.net2_packet_decode_burst_host(ctypes.byref(k), 16, _p(d), _p(o), _p(ln),
                                           4, _p(r), None, None, None, 0) == errno.EINVAL
    k = rx_keys(0, b"", True)
    assert L.net2_packet_decode_burst_host(ctypes.byref(k), 65, _p(d), _p(o), _p(ln),
                                           4, _p(r), None, None, None, 0) == errno.EINVAL
    assert L.net2_packet_decode_burst_host(ctypes.byref(k), 16, _p(d), _p(o), _p(ln),
                                           4, _p(r), None, _p(s), None, 0) == errno.EINVAL
    assert L.net2_packet_decode_burst_host(None, 16, _p(d), _p(o), _p(ln),
                                           4, _p(r), None, None, None, 0) == errno.EINVAL
    assert L.net2_packet_encode_burst_host(6, b"k" * 64, 64, 1, None, _p(s), _p(d),
                                           _p(o), _p(ln), 4, _p(r), 0) == errno.EINVAL
    assert L.net2_packet_encode_burst_host(1, None, 0, 1, _p(s), _p(s), _p(d),
                                           _p(o), _p(ln), 4, _p(r), 0) == errno.EINVAL
    # an empty burst is a no-op
    assert L.net2_packet_decode_burst_host(ctypes.byref(k), 16, None, None, None, 0,
                                           None, None, None, None, 0) == 0
    assert L.net2_packet_encode_burst_host(0, None, 0, 0, None, None, None, None,
                                           None, 0, None, 0) == 0


@pytest.mark.parametrize("gap", [0, 7, 2000])
def test_host_burst_pinned_layouts(dev, oracle_mod, gap):
    """Datagrams in one page-locked arena: back to back or with small gaps
    (dense: copied to the GPU as they lie, no host pack) and with gaps as
    large as the datagrams (sparse: packed into staging) -- the same codes,
    sealed bytes, headers and IVs either way."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(80 + gap)
    n, alg, ivlen = 120_000, 6, 16
    lens = rng.choice(np.array([136, 584, 1500], dtype=np.uint32), n)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gap)
    total = int(offs[-1] + lens[-1])
    buf = pinned((total,), np.uint8)
    buf[:] = rng.integers(0, 256, total, dtype=np.uint8)
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    flags = np.full(n, PH_SIGNED | PH_ENCRYPTED, dtype=np.uint32)
    key = bytes(range(64))
    o_res, o_sealed = oracle_mod.packet_encode_batch(alg, key, True, seq, flags, buf,
                                                     offs, lens, nthreads=CPU_THREADS)
    res = encode_host(L, alg, key, True, seq, flags, buf, offs, lens)
    assert np.array_equal(res, o_res) and (res == OK).all()
    assert np.array_equal(buf, o_sealed)
    bad = np.sort(rng.choice(n, 999, replace=False))
    buf[(offs[bad] + 70).astype(np.int64)] ^= 4      # inside the hash field
    got = decode_host(L, rx_keys(alg, key, True), ivlen, buf, offs, lens)
    want = oracle_mod.packet_decode_batch(alg, key, True, ivlen, buf, offs, lens,
                                          nthreads=CPU_THREADS)
    check_decode(got, want, ivlen)
    assert np.array_equal(np.nonzero(got["res"])[0], bad)


@pytest.mark.parametrize("memory", ["pageable", "pinned"])
def test_host_burst_large_datagrams(dev, oracle_mod, memory):
    """Datagrams up to the UDP maximum (65,507-byte payloads; the reference's
    receive buffer takes whatever one recvfrom returns, src/sockdgram.c:67-108)
    mixed with runts and MTU sizes: ~200 MB, so each 64 MiB chunk holds a few
    thousand datagrams and the burst crosses several chunks in both slots.
    TX then RX (every 50th datagram tampered) against the oracle."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(8081)
    n, alg, ivlen = 12001, 6, 16
    payload = rng.choice(np.array([0, 100, 1428, 9000, 32768, 65507 - 72]), n,
                         p=[0.05, 0.2, 0.25, 0.2, 0.15, 0.15])
    lens = (8 + 64 + payload).astype(np.uint32)
    lens[rng.random(n) < 0.02] = 5                 # runts
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    flags = np.full(n, PH_SIGNED | PH_ENCRYPTED, dtype=np.uint32)
    key = bytes(range(40, 104))
    o_res, o_sealed = oracle_mod.packet_encode_batch(
        alg, key, True, seq, flags, data, offs, lens, nthreads=CPU_THREADS)
    if memory == "pinned":
        buf = pinned(data.shape, np.uint8)
        buf[:] = data
    else:
        buf = data.copy()
    del data
    res = encode_host(L, alg, key, True, seq, flags, buf, offs, lens)
    assert np.array_equal(res, o_res)
    assert np.array_equal(buf, o_sealed)
    del o_sealed
    bad = np.nonzero((np.arange(n) % 50 == 7) & (lens > 72))[0]
    buf[(offs[bad] + 8 + (lens[bad] - 9) // 2).astype(np.int64)] ^= 0x01
    got = decode_host(L, rx_keys(alg, key, True), ivlen, buf, offs, lens)
    want = oracle_mod.packet_decode_batch(alg, key, True, ivlen, buf, offs, lens,
                                          nthreads=CPU_THREADS)
    check_decode(got, want, ivlen)
    assert (got["res"][bad] == BAD).all() and (got["res"] == OK).sum() > n // 2
