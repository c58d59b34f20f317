"""GPU parity on seeded random layouts: many small batches whose shape is
drawn at random -- algorithm, packet count (incl. counts that are not a
multiple of the wave or workgroup size), lengths mixing empty packets, the
SHA256Pad / SHA512Pad boundary lengths (src/sha2.c:495-543, 784-832) and
long packets, packet start alignment (A16 / A4 / A1 address modes), gaps
between packets, binned and unbinned order, plain and keyed (HMAC) rows --
each checked digest-for-digest against the oracle.  Deterministic: every
trial is a pure function of its seed."""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

BOUNDARY = (0, 1, 55, 56, 63, 64, 65, 111, 112, 119, 120, 127, 128, 129)


def _layout(rng):
    n = int(rng.choice([1, 63, 64, 65, 255, 257, 1000, 2049]))
    kind = rng.integers(0, 3)
    if kind == 0:
        lens = rng.choice(BOUNDARY, n)
    elif kind == 1:
        lens = rng.integers(0, 3000, n)
    else:
        lens = np.where(rng.random(n) < 0.9, rng.choice(BOUNDARY, n),
                        rng.integers(3000, 20000, n))
    align = int(rng.choice([1, 4, 16]))
    gap = int(rng.choice([0, 0, 3, 17]))
    return lens.astype(np.uint32), align, gap


def _dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (HIP device not visible)")
    return torch.device("cuda:0")


@pytest.mark.parametrize("seed", range(12))
def test_random_var_layouts(dev, oracle_mod, seed):
    from ilias_net2_amd import batch
    rng = np.random.default_rng(1000 + seed)
    lens, align, gap = _layout(rng)
    alg = int(rng.integers(1, 4))
    data, offs = synth.packed(2000 + seed, lens, align=align, gap=gap)
    want = oracle_mod.batch(alg, data, offsets=offs, lens=lens, nthreads=8)
    for binned in (True, False):
        got = batch.digest_var(alg, _dev(data, dev),
                               _dev(offs.astype(np.int64), dev),
                               _dev(lens.astype(np.int32), dev),
                               binned=binned).cpu().numpy()
        assert np.array_equal(got, want), (seed, alg, align, gap, binned)


@pytest.mark.parametrize("seed", range(8))
def test_random_fixed_layouts(dev, oracle_mod, seed):
    from ilias_net2_amd import batch
    rng = np.random.default_rng(3000 + seed)
    n = int(rng.choice([1, 65, 257, 4097]))
    length = int(rng.choice(list(BOUNDARY) + [1024, 1500, 4096]))
    stride = length + int(rng.choice([0, 1, 4, 12, 16, 64]))
    stride = max(stride, 1)
    alg = int(rng.integers(1, 4))
    data = synth.fixed_batch(4000 + seed, n, length, stride)
    want = oracle_mod.batch(alg, data, stride=stride, length=length, n=n,
                            nthreads=8)
    got = batch.digest_fixed(alg, _dev(data, dev), stride, length, n)
    assert np.array_equal(got.cpu().numpy(), want), (seed, alg, length, stride)


@pytest.mark.parametrize("seed", range(6))
def test_random_hmac_layouts(dev, oracle_mod, seed):
    from ilias_net2_amd import batch
    rng = np.random.default_rng(5000 + seed)
    lens, align, gap = _layout(rng)
    alg = int(rng.integers(4, 7))
    key = bytes(synth.random_bytes(6000 + seed, {4: 32, 5: 48, 6: 64}[alg]))
    data, offs = synth.packed(7000 + seed, lens, align=align, gap=gap)
    want = np.stack([np.frombuffer(oracle_mod.hmac(
        alg, key, data[int(o):int(o) + int(l)].tobytes()), dtype=np.uint8)
        for o, l in zip(offs, lens)])
    got = batch.hmac_dev(alg, key, _dev(data, dev),
                         offsets=_dev(offs.astype(np.int64), dev),
                         lens=_dev(lens.astype(np.int32), dev),
                         binned=bool(seed % 2)).cpu().numpy()
    assert np.array_equal(got, want), (seed, alg, align, gap)


@pytest.mark.parametrize("seed", range(8))
def test_random_sign_verify_layouts(dev, oracle_mod, seed):
    """The datagram authenticator on random layouts (types/packet.n2t:226-257,
    410-427): sign in place, tamper with a few datagrams (in the field or the
    message), verify -- every sealed byte and every verdict against the
    oracle's HMAC, binned and unbinned, at every start alignment (the SHA-256
    sign / verify instances take the pair loop since round 5)."""
    from ilias_net2_amd import batch
    rng = np.random.default_rng(9000 + seed)
    lens, align, gap = _layout(rng)
    alg = int(rng.integers(4, 7))
    dl = {4: 32, 5: 48, 6: 64}[alg]
    lens = (lens + np.where(rng.random(len(lens)) < 0.9, dl, 0)).astype(np.uint32)
    key = bytes(synth.random_bytes(9100 + seed, dl))
    data, offs = synth.packed(9200 + seed, lens, align=align, gap=gap)
    sealed = data.copy()
    for o, l in zip(offs, lens):
        o, l = int(o), int(l)
        if l >= dl:
            sealed[o:o + dl] = np.frombuffer(oracle_mod.hmac(
                alg, key, data[o + dl:o + l].tobytes()), dtype=np.uint8)
    binned = bool(seed % 2)
    d = _dev(data, dev)
    o_t = _dev(offs.astype(np.int64), dev)
    l_t = _dev(lens.astype(np.int32), dev)
    batch.hmac_sign_dev(alg, key, d, o_t, l_t, binned=binned)
    got = d.cpu().numpy()
    assert np.array_equal(got, sealed), (seed, alg, align, gap)
    rx = sealed.copy()
    want = np.where(lens >= dl, 0, 2).astype(np.uint8)
    for i in np.nonzero((rng.random(len(lens)) < 0.1) & (lens > 0))[0]:
        rx[int(offs[i]) + int(rng.integers(0, lens[i]))] ^= 0x08
        if lens[i] >= dl:
            want[i] = 1
    v = batch.hmac_verify_dev(alg, key, _dev(rx, dev), o_t, l_t,
                              binned=binned).cpu().numpy()
    assert np.array_equal(v, want), (seed, alg, align, gap, np.nonzero(v != want)[0][:8])
