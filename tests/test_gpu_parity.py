"""GPU parity: every digest from the HIP path, through the C ABI, equals the
oracle's (bit-exact) on the same seeded inputs.

Covers the reference's own KATs (test/hash.cc), the boundary lengths where
SHA256Pad / SHA512Pad change shape (src/sha2.c:495-543, 784-832), empty and
ragged packets, unaligned packet starts, the length-binned variable path, the
host-memory end-to-end path, and BASELINE.json's configs at full size
(1 M x 1 KiB SHA-256 / SHA-512, 1 M x {64, 512, 1500} B) checked
digest-for-digest against the oracle run on the host cores.
"""
import hashlib
import os

import numpy as np
import pytest

import synth
from golden.make_golden import FIPS_MESSAGES, pattern

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

NAMES = {1: "SHA256", 2: "SHA384", 3: "SHA512"}
CPU_THREADS = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (HIP device not visible)")
    from ilias_net2_amd import _lib
    assert _lib.device_count() >= 1, "no gfx950 device found by the C ABI"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def batch():
    from ilias_net2_amd import batch as b
    return b


@pytest.fixture(scope="module")
def H():
    from ilias_net2_amd import hash as h
    return h


def to_dev(a: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def dd(d: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(d).tobytes()).hexdigest()


# ---- the reference's C++ hash API (test/hash.cc:50-80), on the GPU ------

def test_reference_hash_cc(dev, H, golden):
    ref = golden["kat"]["reference"]
    msg = ref["message"].encode()
    for fac, name in ((H.sha256(), "SHA256"), (H.sha384(), "SHA384"),
                      (H.sha512(), "SHA512")):
        assert fac.run(b"", msg).hex() == ref[name]          # factory.run()
        ctx = fac.instantiate(b"")                             # instantiate
        ctx.update(msg)                                        # update
        assert ctx.final().hex() == ref[name]                  # final


def test_fips_and_boundaries_single(dev, H, golden):
    for key, m in FIPS_MESSAGES.items():
        for alg, name in NAMES.items():
            assert H.hashbuf(alg, b"", m).hex() == golden["kat"]["fips"][key][name]
    for n, row in golden["kat"]["boundary"].items():
        m = pattern(int(n))
        for alg, name in NAMES.items():
            assert H.hashbuf(alg, b"", m).hex() == row[name], (n, name)


def test_sha2c_recorded_outputs(dev, H, golden):
    for n, v in golden["sha2c"]["vectors"].items():
        m = pattern(int(n))
        assert H.hashbuf(1, b"", m).hex() == v["SHA256"]
        assert H.hashbuf(3, b"", m).hex().startswith(v["SHA512_prefix"])


def test_iovec_segments(dev, H):
    """hashbuf over several iovecs == over their concatenation (the
    SHA256Update-per-iovec loop of src/sign.c:298-304)."""
    rng = np.random.default_rng(3)
    m = rng.integers(0, 256, 777, dtype=np.uint8).tobytes()
    segs = [m[:1], m[1:64], b"", m[64:500], m[500:]]
    for alg in NAMES:
        assert H.hashbuf(alg, b"", segs) == H.hashbuf(alg, b"", m)


# ---- device-resident fixed layout -----------------------------------------

def test_golden_batches(dev, batch, golden, oracle_mod):
    for b in golden["batches"]:
        if b["kind"] == "fixed":
            data = synth.fixed_batch(b["seed"], b["n"], b["len"], b["stride"])
            out = batch.digest_fixed(b["alg"], to_dev(data, dev), b["stride"],
                                     b["len"], b["n"]).cpu().numpy()
        else:
            lens = synth.mixed_lengths(b["len_seed"], b["n"])
            data, offs = synth.packed(b["seed"], lens, align=b["align"])
            out = batch.digest_var(b["alg"], to_dev(data, dev),
                                   to_dev(offs.astype(np.int64), dev),
                                   to_dev(lens.astype(np.int32), dev)).cpu().numpy()
        assert dd(out) == b["digest_of_digests"], b
        assert out[0].tobytes().hex() == b["first"]


LENGTHS = [0, 1, 3, 55, 56, 57, 63, 64, 65, 111, 112, 113, 119, 120, 127,
           128, 129, 255, 256, 1000, 1023, 1024, 1500]


@pytest.mark.parametrize("alg", [1, 2, 3])
@pytest.mark.parametrize("stride_kind", ["aligned16", "tight", "odd"])
def test_fixed_lengths(dev, batch, oracle_mod, alg, stride_kind):
    for i, length in enumerate(LENGTHS):
        n = 300 + i  # not a multiple of the 256-lane block
        stride = {"aligned16": (length + 15) // 16 * 16 or 16,
                  "tight": max(length, 1),
                  "odd": length + 3}[stride_kind]
        data = synth.fixed_batch(100 + i, n, length, stride)
        got = batch.digest_fixed(alg, to_dev(data, dev), stride, length,
                                 n).cpu().numpy()
        want = oracle_mod.batch(alg, data, stride=stride, length=length, n=n,
                                nthreads=CPU_THREADS)
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, (alg, stride_kind, length, bad[:8])


def test_fixed_unaligned_base(dev, batch, oracle_mod):
    """A packet batch starting at every byte offset of a dword."""
    for shift in (1, 2, 3, 5, 8):
        length, n = 200, 513
        raw = synth.random_bytes(77 + shift, shift + n * length)
        t = to_dev(raw, dev)[shift:]
        for alg in (1, 3):
            got = batch.digest_fixed(alg, t, length, length, n).cpu().numpy()
            want = oracle_mod.batch(alg, raw[shift:], stride=length,
                                    length=length, n=n)
            assert np.array_equal(got, want), (shift, alg)


def test_single_and_empty(dev, batch, oracle_mod):
    for alg in NAMES:
        t = torch.zeros(16, dtype=torch.uint8, device=dev)
        got = batch.digest_fixed(alg, t, 16, 0, 1).cpu().numpy()
        assert got[0].tobytes() == oracle_mod.digest(alg, b"")
        t = to_dev(np.frombuffer(b"abc", dtype=np.uint8), dev)
        got = batch.digest_fixed(alg, t, 3, 3, 1).cpu().numpy()
        assert got[0].tobytes() == oracle_mod.digest(alg, b"abc")


def test_max_payload(dev, batch, oracle_mod):
    """65,536-byte payloads, the 16-bit carver limit (src/carver.c:150,161)."""
    n, length = 130, 65536
    data = synth.fixed_batch(5, n, length)
    for alg in NAMES:
        got = batch.digest_fixed(alg, to_dev(data, dev), length, length,
                                 n).cpu().numpy()
        want = oracle_mod.batch(alg, data, stride=length, length=length, n=n,
                                nthreads=CPU_THREADS)
        assert np.array_equal(got, want), alg


# ---- device-resident variable layout (length-binned) ---------------------

@pytest.mark.parametrize("alg", [1, 2, 3])
@pytest.mark.parametrize("align", [1, 4, 16])
def test_var_ragged(dev, batch, oracle_mod, alg, align):
    rng = np.random.default_rng(alg * 31 + align)
    n = 5000
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    lens[:40] = np.array(LENGTHS + LENGTHS[:17], dtype=np.uint32)
    data, offs = synth.packed(1000 + alg, lens, align=align, gap=1)
    want = oracle_mod.batch(alg, data, offsets=offs, lens=lens,
                            nthreads=CPU_THREADS)
    dt = to_dev(data, dev)
    do = to_dev(offs.astype(np.int64), dev)
    dl = to_dev(lens.astype(np.int32), dev)
    for binned in (True, False):
        got = batch.digest_var(alg, dt, do, dl, binned=binned).cpu().numpy()
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, (binned, bad[:8])


def test_var_permuted_offsets(dev, batch, oracle_mod):
    """Offsets need not be sorted or disjoint: shuffled and repeated packets."""
    rng = np.random.default_rng(9)
    lens0 = synth.mixed_lengths(9, 3000)
    data, offs0 = synth.packed(10, lens0)
    idx = rng.integers(0, 3000, 7000)
    offs, lens = offs0[idx], lens0[idx]
    want = oracle_mod.batch(1, data, offsets=offs, lens=lens)
    got = batch.digest_var(1, to_dev(data, dev), to_dev(offs.astype(np.int64), dev),
                           to_dev(lens.astype(np.int32), dev)).cpu().numpy()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("alg", [1, 2, 3])
@pytest.mark.parametrize("align", [16, 4, 1])
def test_var_whole_block_lengths(dev, batch, oracle_mod, alg, align):
    """Lanes that share one whole-block length read the pad block's schedule
    from the kernels' constant tables (g_padtab256 per wave, g_padtab512 per
    workgroup): both ends of each table, one past it, in each address mode
    (16-byte, 4-byte and byte-aligned packet starts), for the digests and the
    HMAC rows (inner length = key block + message)."""
    if alg == 1:
        blk, js, copies = 64, (0, 1, 2, 8, 1023, 1024, 1025, 1026), 70
    else:   # SHA-384/512: whole 256-lane workgroups of one length
        blk, js, copies = 128, (0, 1, 2, 8, 511, 512, 513, 514), 520
    lens = np.repeat(np.array([blk * j for j in js], dtype=np.uint32), copies)
    lens = np.concatenate([lens, np.array([blk, blk - 4, 0, 3], dtype=np.uint32)])
    data, offs = synth.packed(77 + align, lens, align=align,
                              gap={16: 0, 4: 4, 1: 1}[align])
    dt = to_dev(data, dev)
    do = to_dev(offs.astype(np.int64), dev)
    dl = to_dev(lens.astype(np.int32), dev)
    want = oracle_mod.batch(alg, data, offsets=offs, lens=lens,
                            nthreads=CPU_THREADS)
    for binned in (True, False):
        got = batch.digest_var(alg, dt, do, dl, binned=binned).cpu().numpy()
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, (binned, lens[bad[:8]])
    halg = alg + 3
    key = bytes(synth.random_bytes(78, DLEN_OF[halg]))
    want = np.stack([np.frombuffer(oracle_mod.hmac(
        halg, key, data[int(o):int(o) + int(l)].tobytes()), dtype=np.uint8)
        for o, l in zip(offs, lens)])
    for binned in (True, False):
        got = batch.hmac_dev(halg, key, dt, offsets=do, lens=dl,
                             binned=binned).cpu().numpy()
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, (binned, lens[bad[:8]])


DLEN_OF = {4: 32, 5: 48, 6: 64}


# ---- host-memory end-to-end path (net2_sha2_batch) ------------------------

def test_host_batch(dev, batch, oracle_mod):
    data = synth.fixed_batch(21, 20000, 1024)
    got = batch.digest_host(1, data, stride=1024, length=1024, n=20000)
    want = oracle_mod.batch(1, data, stride=1024, length=1024, n=20000,
                            nthreads=CPU_THREADS)
    assert np.array_equal(got, want)
    # padded stride, last packet ends exactly at the buffer end
    n, length, stride = 999, 100, 128
    data = synth.random_bytes(22, (n - 1) * stride + length)
    got = batch.digest_host(3, data, stride=stride, length=length, n=n)
    want = oracle_mod.batch(3, data, stride=stride, length=length, n=n)
    assert np.array_equal(got, want)
    # pinned (page-locked) source and destination: direct DMA path
    n, length, stride = 70001, 1000, 1008
    src = torch.from_numpy(synth.random_bytes(25, (n - 1) * stride + length)).pin_memory()
    out = torch.empty((n, 32), dtype=torch.uint8).pin_memory()
    from ilias_net2_amd import _lib
    rc = _lib.lib().net2_sha2_batch(1, src.data_ptr(), None, None, stride,
                                    length, n, out.data_ptr(), 0)
    assert rc == 0
    want = oracle_mod.batch(1, src.numpy(), stride=stride, length=length, n=n,
                            nthreads=CPU_THREADS)
    assert np.array_equal(out.numpy(), want)
    # variable layout, unaligned
    lens = synth.mixed_lengths(23, 30000)
    data, offs = synth.packed(24, lens)
    got = batch.digest_host(2, data, offsets=offs, lens=lens)
    want = oracle_mod.batch(2, data, offsets=offs, lens=lens,
                            nthreads=CPU_THREADS)
    assert np.array_equal(got, want)


def test_host_batch_digests_to_mapped_memory(dev, batch, oracle_mod):
    """The host path stores digests straight into pinned host memory through
    its device mapping: registered (hipHostRegister) memory at an interior,
    odd offset; the variable layout into pinned memory; and the D2H-copy
    fallback of the same calls in a child process (NET2_SHA2_D2H_COPY=1)."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    n, length = 30000, 700
    data = synth.random_bytes(31, n * length)
    want = oracle_mod.batch(3, data, stride=length, length=length, n=n,
                            nthreads=CPU_THREADS)
    # a registered page-aligned buffer; digests written from byte 13 on
    buf = np.zeros(n * 64 + 8192, dtype=np.uint8)
    base = buf.ctypes.data
    a0 = (base + 4095) & ~4095
    span = n * 64 + 4096
    cr = torch.cuda.cudart()
    assert int(cr.cudaHostRegister(a0, span, 0)) == 0
    try:
        at = a0 + 13
        rc = L.net2_sha2_batch(3, data.ctypes.data, None, None, length, length,
                               n, at, 1)
        assert rc == 0
        got = buf[at - base: at - base + n * 64].reshape(n, 64)
        assert np.array_equal(got, want)
        assert not buf[:at - base].any()          # nothing outside the range
        assert not buf[at - base + n * 64:].any()
    finally:
        assert int(cr.cudaHostUnregister(a0)) == 0
    # variable layout (binned, scattered digest stores) into pinned memory
    lens = synth.mixed_lengths(32, 40000)
    data, offs = synth.packed(33, lens)
    out = torch.zeros((len(lens), 32), dtype=torch.uint8).pin_memory()
    o64 = np.ascontiguousarray(offs, dtype=np.uint64)   # kept alive for the call
    l32 = np.ascontiguousarray(lens, dtype=np.uint32)
    rc = L.net2_sha2_batch(1, data.ctypes.data, o64.ctypes.data, l32.ctypes.data,
                           0, 0, len(lens), out.data_ptr(), 1)
    assert rc == 0
    assert np.array_equal(out.numpy(), oracle_mod.batch(1, data, offsets=offs, lens=lens,
                                                        nthreads=CPU_THREADS))


def test_host_batch_d2h_copy_fallback(dev):
    """NET2_SHA2_D2H_COPY=1 (the D2H-copy form, kept for A/B) gives the same
    digests as the default form, pinned and pageable outputs alike."""
    import subprocess
    import sys
    code = r'''
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np
import torch
import synth
from oracle import oracle
from ilias_net2_amd import batch, _lib
data = synth.fixed_batch(34, 20000, 1024)
want = oracle.batch(1, data, stride=1024, length=1024, n=20000, nthreads=4)
assert np.array_equal(batch.digest_host(1, data, stride=1024, length=1024, n=20000), want)
out = torch.empty((20000, 32), dtype=torch.uint8).pin_memory()
assert _lib.lib().net2_sha2_batch(1, data.ctypes.data, None, None, 1024, 1024, 20000,
                                  out.data_ptr(), 1) == 0
assert np.array_equal(out.numpy(), want)
print("ok")
'''
    import os
    env = dict(os.environ, NET2_SHA2_D2H_COPY="1")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_host_batch_var_multichunk(dev, batch, oracle_mod):
    """Variable layout from pageable memory over several 64 MiB chunks whose
    byte and packet counts differ (staging growth, parallel gather), twice
    so the second call reuses the grown staging buffers."""
    lens = synth.mixed_lengths(26, 200000, choices=(64, 512, 1500, 1472, 20, 9000))
    data, offs = synth.packed(27, lens, align=4, gap=3)
    want = oracle_mod.batch(1, data, offsets=offs, lens=lens,
                            nthreads=CPU_THREADS)
    for _ in range(2):
        got = batch.digest_host(1, data, offsets=offs, lens=lens, max_devices=1)
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, bad[:8]


def test_host_batch_skewed_chunks(dev, batch, oracle_mod):
    """Chunks are cut by packet count at the slice's mean size: a run of
    jumbo packets ahead of many runts puts ~2x kChunkBytes in the first
    chunk (staging grows to fit).  Also a pageable fixed layout whose stride
    is not the 16-byte padded length (parallel strided gather, two chunks)."""
    lens = np.concatenate([np.full(15000, 9000), np.full(150000, 20)]).astype(np.uint32)
    data, offs = synth.packed(28, lens, align=1, gap=1)
    got = batch.digest_host(1, data, offsets=offs, lens=lens, max_devices=1)
    want = oracle_mod.batch(1, data, offsets=offs, lens=lens,
                            nthreads=CPU_THREADS)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, bad[:8]
    n, length, stride = 70000, 1000, 1001
    data = synth.random_bytes(29, (n - 1) * stride + length)
    got = batch.digest_host(3, data, stride=stride, length=length, n=n,
                            max_devices=1)
    want = oracle_mod.batch(3, data, stride=stride, length=length, n=n,
                            nthreads=CPU_THREADS)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, bad[:8]


# ---- BASELINE.json configs at full size ------------------------------------

def _full_fixed(dev, batch, oracle_mod, alg, seed):
    n, length = 1 << 20, 1024
    data = synth.fixed_batch(seed, n, length)
    got = batch.digest_fixed(alg, to_dev(data, dev), length, length,
                             n).cpu().numpy()
    want = oracle_mod.batch(alg, data, stride=length, length=length, n=n,
                            nthreads=CPU_THREADS)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, bad[:8]


def test_config2_full_sha256(dev, batch, oracle_mod):
    _full_fixed(dev, batch, oracle_mod, 1, 2)


def test_config4_full_sha512(dev, batch, oracle_mod):
    _full_fixed(dev, batch, oracle_mod, 3, 5)


@pytest.mark.parametrize("alg", [1, 2, 3])
def test_config3_full_mixed(dev, batch, oracle_mod, alg):
    """C3 at full size, and the same mix through SHA-384 / SHA-512 (the
    c3_512 bench config)."""
    n = 1 << 20
    lens = synth.mixed_lengths(3, n)
    data, offs = synth.packed(4, lens)
    got = batch.digest_var(alg, to_dev(data, dev), to_dev(offs.astype(np.int64), dev),
                           to_dev(lens.astype(np.int32), dev)).cpu().numpy()
    want = oracle_mod.batch(alg, data, offsets=offs, lens=lens,
                            nthreads=CPU_THREADS)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, bad[:8]


def test_repeat_is_deterministic(dev, batch):
    data = to_dev(synth.fixed_batch(1, 4096, 1024), dev)
    a = batch.digest_fixed(1, data, 1024, 1024, 4096)
    b = batch.digest_fixed(1, data, 1024, 1024, 4096)
    assert torch.equal(a, b)


# ---- HMAC rows ------------------------------------------

def test_hmac_single(dev, H, golden):
    """net2_hashctx_hashiov on keyed rows == the golden HMAC vectors
    (oracle + Python hmac agree on them)."""
    facs = {4: H.hmac_sha256(), 5: H.hmac_sha384(), 6: H.hmac_sha512()}
    for v in golden["kat"]["hmac"]:
        key = bytes.fromhex(v["key"])
        assert facs[v["alg"]].run(key, pattern(v["len"])).hex() == v["digest"]
        ctx = facs[v["alg"]].instantiate(key)
        ctx.update(pattern(v["len"]))
        assert ctx.final().hex() == v["digest"]


@pytest.mark.parametrize("alg", [4, 5, 6])
def test_hmac_batches(dev, batch, oracle_mod, alg):
    import hmac as pyhmac
    hl = {4: 32, 5: 48, 6: 64}[alg]
    key = bytes(synth.random_bytes(40 + alg, hl))
    # fixed layout across the padding boundaries; strides that put every
    # packet on a 16-byte (A16), 4-byte (A4) or odd (A1) address; lengths
    # that are block multiples take the constant-pad-block kernel
    for length in (0, 1, 55, 56, 64, 111, 112, 128, 1000, 1024):
        n = 257
        for stride in (length + 5, max(16, -(-length // 16) * 16),
                       -(-length // 4) * 4 + 4):
            data = synth.fixed_batch(50 + length, n, length, stride)
            got = batch.hmac_dev(alg, key, to_dev(data, dev), stride=stride,
                                 length=length, n=n).cpu().numpy()
            for i in range(n):
                msg = data[i * stride:i * stride + length].tobytes()
                assert got[i].tobytes() == oracle_mod.hmac(alg, key, msg), (length, stride, i)
        h = {4: "sha256", 5: "sha384", 6: "sha512"}[alg]
        msg = data[:length].tobytes()
        assert got[0].tobytes() == pyhmac.new(key, msg, h).digest()
    # variable layout (MTU-sized datagrams), binned and not
    lens = synth.mixed_lengths(60 + alg, 3000, choices=(64, 512, 1500, 1472, 20))
    data, offs = synth.packed(61 + alg, lens)
    want = np.stack([np.frombuffer(oracle_mod.hmac(
        alg, key, data[int(o):int(o) + int(l)].tobytes()), dtype=np.uint8)
        for o, l in zip(offs, lens)])
    for binned in (True, False):
        got = batch.hmac_dev(alg, key, to_dev(data, dev),
                             offsets=to_dev(offs.astype(np.int64), dev),
                             lens=to_dev(lens.astype(np.int32), dev),
                             binned=binned).cpu().numpy()
        assert np.array_equal(got, want), binned


# ---- net2_ph_to_iv (types/packet.n2t:100-158) -------------

def test_ph_to_iv(dev, oracle_mod):
    import ctypes
    from ilias_net2_amd import _lib
    L = _lib.lib()

    class PH(ctypes.Structure):
        _fields_ = [("seq", ctypes.c_uint32), ("flags", ctypes.c_uint32)]
    # single-header form, any ivlen (the reference loop)
    for seq, flags in ((0, 0), (1, 2), (0xFFFFFFFF, 0x80000001)):
        for ivlen in (0, 1, 16, 31, 32, 33, 64, 65, 100):
            out = ctypes.create_string_buffer(max(ivlen, 1))
            assert L.net2_ph_to_iv_buf(ctypes.byref(PH(seq, flags)), ivlen, out) == 0
            assert out.raw[:ivlen] == oracle_mod.ph_to_iv(seq, flags, ivlen)
    # batched device form
    n = 100003
    rng = np.random.default_rng(17)
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    flags = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ds = to_dev(seq.view(np.int32), dev)
    df = to_dev(flags.view(np.int32), dev)
    for ivlen in (16, 32, 48, 64):
        out = torch.empty(n * ivlen, dtype=torch.uint8, device=dev)
        rc = L.net2_ph_to_iv_dev(ds.data_ptr(), df.data_ptr(), n, ivlen,
                                 out.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        got = out.cpu().numpy().reshape(n, ivlen)
        for i in list(range(0, n, 997)) + [n - 1]:
            assert got[i].tobytes() == oracle_mod.ph_to_iv(int(seq[i]), int(flags[i]), ivlen), (ivlen, i)
    out = torch.empty(65, dtype=torch.uint8, device=dev)
    assert L.net2_ph_to_iv_dev(ds.data_ptr(), df.data_ptr(), 1, 65,
                               out.data_ptr(), None) == 22  # EINVAL above 64


# ---- host threading and graph capture (include/net2/sha2_batch.h) -------------

def test_concurrent_host_threads(dev, H, oracle_mod):
    """Callers are threadpool workers in the reference (threadpool.h:33-34):
    many threads calling hashbuf / net2_sha2_batch at once."""
    import threading
    from ilias_net2_amd import batch
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(t)
            for j in range(20):
                m = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
                alg = 1 + (t + j) % 3
                if H.hashbuf(alg, b"", m) != oracle_mod.digest(alg, m):
                    errors.append(("hashbuf", t, j))
            data = synth.fixed_batch(500 + t, 3000, 700)
            got = batch.digest_host(1 + t % 3, data, stride=700, length=700, n=3000)
            if not np.array_equal(got, oracle_mod.batch(1 + t % 3, data, stride=700,
                                                        length=700, n=3000)):
                errors.append(("batch", t))
        except Exception as e:  # noqa: BLE001
            errors.append(("exc", t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:5]


def test_concurrent_streams_device_paths(dev, batch, oracle_mod):
    """Device-resident batches submitted from several host threads at once,
    each on its own stream with its own workspace and outputs (the way a
    multi-stream caller overlaps batches): binned variable-length digests,
    HMAC over a fixed layout and a packet burst round trip, ten times each
    per thread, every result checked."""
    import ctypes
    import threading
    from ilias_net2_amd import _lib
    L = _lib.lib()
    n = 20000
    jobs = []
    for t in range(4):
        lens = synth.mixed_lengths(900 + t, n)
        data, offs = synth.packed(910 + t, lens, align=1 + 3 * (t % 2))
        alg = 1 + t % 3
        fdata = synth.fixed_batch(920 + t, n, 700)
        key = bytes(synth.random_bytes(930 + t, 64))
        jobs.append(dict(
            alg=alg, vd=to_dev(data, dev), vo=to_dev(offs.astype(np.int64), dev),
            vl=to_dev(lens.astype(np.int32), dev),
            want_v=oracle_mod.batch(alg, data, offsets=offs, lens=lens,
                                    nthreads=CPU_THREADS),
            fd=to_dev(fdata, dev), key=key,
            want_h=np.stack([np.frombuffer(oracle_mod.hmac(
                6, key, fdata[i * 700:(i + 1) * 700].tobytes()), dtype=np.uint8)
                for i in range(0, n, 97)])))
    errors = []

    def worker(t):
        try:
            j = jobs[t]
            s = torch.cuda.Stream(dev)
            ws = batch.var_workspace(n, dev, stream=s)
            bws = torch.empty(L.net2_packet_burst_workspace(n), dtype=torch.uint8,
                              device=dev)
            for r in range(10):
                with torch.cuda.stream(s):
                    got = batch.digest_var(j["alg"], j["vd"], j["vo"], j["vl"],
                                           workspace=ws, stream=s)
                    hm = batch.hmac_dev(6, j["key"], j["fd"], stride=700,
                                        length=700, n=n, stream=s)
                    # burst: seal a copy of the variable batch, then open it
                    d = j["vd"].clone()
                    seq = torch.arange(n, dtype=torch.int32, device=dev) + r
                    fl = torch.full((n,), 3, dtype=torch.int32, device=dev)
                    res = torch.full((n,), 9, dtype=torch.uint8, device=dev)
                    rc1 = L.net2_packet_encode_burst(
                        6, j["key"], 64, 1, seq.data_ptr(), fl.data_ptr(),
                        d.data_ptr(), j["vo"].data_ptr(), j["vl"].data_ptr(), n,
                        res.data_ptr(), bws.data_ptr(), bws.numel(), s.cuda_stream)
                    enc = res.clone()
                    rc2 = L.net2_packet_decode_burst(
                        6, j["key"], 64, 1, 0, d.data_ptr(), j["vo"].data_ptr(),
                        j["vl"].data_ptr(), n, res.data_ptr(), None, None, None,
                        bws.data_ptr(), bws.numel(), s.cuda_stream)
                s.synchronize()
                if rc1 or rc2:
                    errors.append(("rc", t, r, rc1, rc2))
                if not np.array_equal(got.cpu().numpy(), j["want_v"]):
                    errors.append(("var", t, r))
                if not np.array_equal(hm.cpu().numpy()[::97], j["want_h"]):
                    errors.append(("hmac", t, r))
                # every slot with room seals (the 64-byte ones have none for
                # header and hash field), and every sealed one opens
                room = j["vl"] >= 8 + 64
                if not (torch.equal(enc[room], torch.zeros_like(enc[room])) and
                        bool((enc[~room] == 1).all()) and
                        torch.equal(res[room], enc[room])):
                    errors.append(("burst", t, r))
        except Exception as e:  # noqa: BLE001
            errors.append(("exc", t, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:5]


def test_graph_capture(dev, batch, oracle_mod):
    """The device entry points allocate and synchronise nothing, so a batch
    launch can be captured into a hipGraph and replayed."""
    n, length = 5000, 1024
    data = to_dev(synth.fixed_batch(77, n, length), dev)
    lens = synth.mixed_lengths(78, n)
    vdata, offs = synth.packed(79, lens)
    vd, vo, vl = to_dev(vdata, dev), to_dev(offs.astype(np.int64), dev), to_dev(lens.astype(np.int32), dev)
    out = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    vout = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    ws = batch.var_workspace(n, dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):  # warm-up outside capture
        batch.digest_fixed(1, data, length, length, n, out=out, stream=s)
        batch.digest_var(3, vd, vo, vl, out=vout, workspace=ws, stream=s)
    torch.cuda.synchronize()
    out.zero_()
    vout.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        batch.digest_fixed(1, data, length, length, n, out=out, stream=s)
        batch.digest_var(3, vd, vo, vl, out=vout, workspace=ws, stream=s)
    g.replay()
    torch.cuda.synchronize()
    want = oracle_mod.batch(1, data.cpu().numpy(), stride=length, length=length, n=n)
    assert np.array_equal(out.cpu().numpy(), want)
    assert np.array_equal(vout.cpu().numpy(), oracle_mod.batch(3, vdata, offsets=offs, lens=lens))


def _hmac_by_composition(batch, alg, key, data, offs, lens, n, dev):
    """RFC 2104 spelled out with the plain digest kernels: inner =
    H((K' ^ ipad) || m) over a rebuilt variable layout, outer =
    H((K' ^ opad) || inner) over a fixed one -- a path independent of the
    HMAC kernel's midstates."""
    halg = alg - 3
    blk = 64 if halg == 1 else 128
    dl = {1: 32, 2: 48, 3: 64}[halg]
    kp = torch.zeros(blk, dtype=torch.uint8, device=dev)
    kp[:len(key)] = torch.tensor(list(key), dtype=torch.uint8, device=dev)
    lens64 = lens.to(torch.int64)
    total = int(lens64.sum())
    owner = torch.repeat_interleave(torch.arange(n, device=dev), lens64)
    start = torch.zeros(n, dtype=torch.int64, device=dev)
    start[1:] = torch.cumsum(lens64, 0)[:-1]
    within = torch.arange(total, device=dev) - start[owner]
    src = offs[owner] + within
    ioffs = start + blk * torch.arange(n, device=dev)
    inner_in = torch.empty(total + blk * n, dtype=torch.uint8, device=dev)
    inner_in[ioffs[owner] + blk + within] = data[src]
    kpos = (ioffs[:, None] + torch.arange(blk, device=dev)[None, :]).reshape(-1)
    inner_in[kpos] = (kp ^ 0x36).repeat(n)
    inner = batch.digest_var(halg, inner_in, ioffs, (lens64 + blk).to(torch.int32))
    outer_in = torch.cat([(kp ^ 0x5c).repeat(n, 1), inner[:, :dl]], dim=1).contiguous()
    return batch.digest_fixed(halg, outer_in.reshape(-1), blk + dl, blk + dl, n)


@pytest.mark.parametrize("alg", [4, 6])
@pytest.mark.parametrize("layout", ["fixed_1k", "mtu_mix"])
def test_hmac_full_size_by_composition(dev, batch, oracle_mod, alg, layout):
    """The HMAC bench configs at full size (1 M x 1 KiB, 1 M x {64, 512,
    1500} B): every digest against the oracle's threaded HMAC batch
    (oracle_hmac_batch, RFC 2104 over the restated src/sha2.c); also
    against RFC 2104 composed from the plain digest kernels (a second,
    GPU-side path independent of the HMAC kernel's midstates)."""
    n = 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(70 + alg)
    if layout == "fixed_1k":
        lens = torch.full((n,), 1024, dtype=torch.int64, device=dev)
    else:
        ch = torch.tensor([64, 512, 1500], dtype=torch.int64, device=dev)
        lens = ch[torch.randint(0, 3, (n,), device=dev, generator=g)]
    offs = torch.zeros(n, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)[:-1]
    data = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8,
                         device=dev, generator=g)
    key = bytes(synth.random_bytes(75 + alg, {4: 32, 6: 64}[alg]))
    if layout == "fixed_1k":
        got = batch.hmac_dev(alg, key, data, stride=1024, length=1024, n=n)
    else:
        got = batch.hmac_dev(alg, key, data, offsets=offs,
                             lens=lens.to(torch.int32))
    offs_h, lens_h = offs.cpu().numpy(), lens.cpu().numpy()
    want_o = oracle_mod.hmac_batch(alg, key, data.cpu().numpy(), offsets=offs_h,
                                   lens=lens_h, nthreads=CPU_THREADS)
    got_h = got.cpu().numpy()
    bad = np.nonzero((got_h != want_o).any(axis=1))[0]
    assert len(bad) == 0, bad[:8]
    want = _hmac_by_composition(batch, alg, key, data, offs,
                                lens.to(torch.int32), n, dev)
    assert torch.equal(got, want)
