"""GPU parity of the datagram authenticator on both sides of the wire
(types/packet.n2t): TX prepends HMAC(key, message) to each datagram
(net2_packet_encode, :410-427) -> net2_hmac_sign_dev; RX removes the first
hashlen bytes as the supplied hash and compares it with the HMAC of the
rest (net2_packet_decode, :226-257) -> net2_hmac_verify_dev.  Checked
against the oracle's HMAC, with tampered messages, tampered hash fields and
datagrams shorter than the hash (NET2_PDECODE_BAD at :240-244 / :254-256)."""
import os

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HL = {4: 32, 5: 48, 6: 64}
CPU_THREADS = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (HIP device not visible)")
    return torch.device("cuda:0")


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _layout(alg, seed, n=3001, align=None):
    rng = np.random.default_rng(seed)
    hl = HL[alg]
    msg = rng.choice([0, 1, 55, 56, 64, 111, 112, 128, 500, 1400, 1500 - hl], n)
    lens = (msg + hl).astype(np.uint32)
    short = rng.random(n) < 0.02                 # runts: shorter than the hash
    lens[short] = rng.integers(0, hl, short.sum()).astype(np.uint32)
    if align is None:
        align = int(rng.choice([1, 4, 16]))
    data, offs = synth.packed(seed + 1, lens, align=align, gap=int(seed % 3))
    return data, offs, lens, short


@pytest.mark.parametrize("alg", [4, 5, 6])
@pytest.mark.parametrize("binned", [True, False])
@pytest.mark.parametrize("align", [1, 4, 16])
def test_sign_then_verify(dev, oracle_mod, alg, binned, align):
    """Every datagram start alignment: the RX compare reads the hash field as
    16-byte vectors, dwords or bytes accordingly."""
    from ilias_net2_amd import batch
    hl = HL[alg]
    key = bytes(synth.random_bytes(80 + alg, hl))
    data, offs, lens, short = _layout(alg, 100 + alg, align=align)
    d = _t(data, dev)
    do, dl = _t(offs.astype(np.int64), dev), _t(lens.astype(np.int32), dev)
    batch.hmac_sign_dev(alg, key, d, do, dl, binned=binned)
    signed = d.cpu().numpy()
    for i, (o, l) in enumerate(zip(offs.astype(np.int64), lens.astype(np.int64))):
        if short[i]:
            assert np.array_equal(signed[o:o + l], data[o:o + l]), i
            continue
        m = data[o + hl:o + l].tobytes()
        assert signed[o:o + hl].tobytes() == oracle_mod.hmac(alg, key, m), i
        assert np.array_equal(signed[o + hl:o + l], data[o + hl:o + l]), i
    # RX: intact datagrams verify, tampered ones do not, runts are flagged
    rng = np.random.default_rng(200 + alg)
    rx = signed.copy()
    want = np.where(short, 2, 0).astype(np.uint8)
    for i in rng.choice(len(lens), 200, replace=False):
        o, l = int(offs[i]), int(lens[i])
        if short[i] or l == 0:
            continue
        pos = o + int(rng.integers(0, l))      # hash field or message byte
        rx[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
        want[i] = 1
    got = batch.hmac_verify_dev(alg, key, _t(rx, dev), do, dl,
                                binned=binned).cpu().numpy()
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    # a different key fails every full-size datagram
    bad = bytes(b ^ 0xFF for b in key)
    got = batch.hmac_verify_dev(alg, bad, _t(signed, dev), do, dl,
                                binned=binned).cpu().numpy()
    assert np.array_equal(got, np.where(short, 2, 1).astype(np.uint8))


def test_dgram_argument_errors(dev):
    from ilias_net2_amd import _lib
    L = _lib.lib()
    t = torch.zeros(64, dtype=torch.uint8, device=dev)
    o = torch.zeros(1, dtype=torch.int64, device=dev)
    n = torch.full((1,), 64, dtype=torch.int32, device=dev)
    key = b"\x00" * 32
    import errno
    # unkeyed row, wrong key length, missing layout arrays
    assert L.net2_hmac_sign_dev(1, key, 32, t.data_ptr(), o.data_ptr(),
                                n.data_ptr(), 1, None, 0, None) == errno.EINVAL
    assert L.net2_hmac_sign_dev(4, key, 31, t.data_ptr(), o.data_ptr(),
                                n.data_ptr(), 1, None, 0, None) == errno.EINVAL
    assert L.net2_hmac_verify_dev(4, key, 32, t.data_ptr(), None,
                                  n.data_ptr(), 1, t.data_ptr(), None, 0,
                                  None) == errno.EINVAL
    assert L.net2_hmac_verify_dev(4, key, 32, t.data_ptr(), o.data_ptr(),
                                  n.data_ptr(), 1, None, None, 0,
                                  None) == errno.EINVAL
    # empty batches are no-ops
    assert L.net2_hmac_sign_dev(4, key, 32, None, None, None, 0, None, 0,
                                None) == 0


@pytest.mark.parametrize("alg", [4, 6])
def test_sign_then_verify_full_size(dev, oracle_mod, alg):
    """The verify bench configs at full size (1 M datagrams, hash field ||
    {64, 512, 1500 - hashlen} B message): every hash field the GPU signed
    equals the oracle's HMAC of its message (oracle_hmac_batch), sign then
    verify accepts every datagram, and one flipped bit in a chosen set of
    datagrams fails exactly those -- the verdicts compared with the
    oracle's own compare of every datagram."""
    from ilias_net2_amd import batch
    n, hl = 1 << 20, HL[alg]
    g = torch.Generator(device=dev)
    g.manual_seed(50 + alg)
    choice = torch.tensor([hl + 64, hl + 512, 1500], dtype=torch.int64, device=dev)
    lens = choice[torch.randint(0, 3, (n,), device=dev, generator=g)]
    offs = torch.zeros(n, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)[:-1]
    d = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8, device=dev,
                      generator=g)
    dl = lens.to(torch.int32)
    key = bytes(synth.random_bytes(90 + alg, hl))
    batch.hmac_sign_dev(alg, key, d, offs, dl)
    assert int(batch.hmac_verify_dev(alg, key, d, offs, dl).sum()) == 0
    rng = np.random.default_rng(60 + alg)
    offs_h, lens_h = offs.cpu().numpy(), lens.cpu().numpy()
    dh = d.cpu().numpy()
    # every hash field against the oracle's HMAC of its message
    want_f = oracle_mod.hmac_batch(alg, key, dh, offsets=offs_h + hl,
                                   lens=lens_h - hl, nthreads=CPU_THREADS)
    fields = dh[offs_h[:, None] + np.arange(hl)[None, :]]
    diff = np.nonzero((fields != want_f).any(axis=1))[0]
    assert len(diff) == 0, diff[:8]
    bad = np.sort(rng.choice(n, 4096, replace=False))
    pos = offs_h[bad] + rng.integers(0, lens_h[bad])
    t = d.clone()
    t[torch.from_numpy(pos.astype(np.int64)).to(dev)] ^= 0x04
    got = batch.hmac_verify_dev(alg, key, t, offs, dl).cpu().numpy()
    # the oracle's verdict for every datagram: field == HMAC(message)
    th = t.cpu().numpy()
    calc = oracle_mod.hmac_batch(alg, key, th, offsets=offs_h + hl,
                                 lens=lens_h - hl, nthreads=CPU_THREADS)
    tf = th[offs_h[:, None] + np.arange(hl)[None, :]]
    want = (tf != calc).any(axis=1).astype(np.uint8)
    assert np.array_equal(got, want)
    assert np.array_equal(np.nonzero(want)[0], bad)
