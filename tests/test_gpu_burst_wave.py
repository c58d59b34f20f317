"""The wave form of the keyed packet bursts (burst_wave_kernel: 1 to 16
datagrams per workgroup, the message schedules expanded by the wave's lanes,
codes / headers / IVs stored by the one launch), which
net2_packet_{decode,encode}_burst[_host] take for bursts of at most 16
datagrams per SIMD (net2_burst_wave_max).

Every parity test of the lane form is run again in the wave form
(net2_sha2_burst_limits raises the limit so bursts of any size take it): the
device-resident bursts of tests/test_gpu_packet.py (six key set-ups, mixed
and wrong flags, slots without room, runts, tampered bytes, the alternate rx
key of net2_ck_rx_key), and the host bursts of tests/test_gpu_burst_host.py
(sliced over 1 and 3 devices, key rollover, pinned layouts, datagrams up to
the UDP maximum -- 512 SHA-512 blocks, 128 passes of 4 blocks at 12
datagrams per workgroup).
Then the default threshold itself at integration-sized bursts, and the two
forms against each other byte for byte.
"""
import os

import numpy as np
import pytest

import test_gpu_burst_host as H
import test_gpu_packet as P

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CPU_THREADS = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a GPU (HIP device not visible)")
    from ilias_net2_amd import _lib
    assert _lib.device_count() >= 1
    return torch.device("cuda:0")


@pytest.fixture
def wave():
    """Every keyed burst of the test in the wave form."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    assert L.net2_sha2_burst_limits(1 << 30, -1) == 0
    yield
    L.net2_sha2_burst_limits(-1, -1)


@pytest.fixture
def virtual(monkeypatch):
    def set_k(k):
        monkeypatch.setenv("NET2_SHA2_VIRTUAL_DEVICES", str(k))
        monkeypatch.setenv("NET2_SHA2_SLICE_MIN_BYTES", "0")
    yield set_k


@pytest.mark.parametrize("hash_alg,enc_set,ivlen", [s for s in P.SETUPS if s[0]])
def test_device_bursts_wave_form(dev, oracle_mod, wave, hash_alg, enc_set, ivlen):
    P.test_encode_then_decode_burst(dev, oracle_mod, hash_alg, enc_set, ivlen)


@pytest.mark.parametrize("hash_alg,no_cutoff", [(6, False), (6, True), (4, False),
                                                (5, False)])
def test_device_alternate_key_wave_form(dev, oracle_mod, wave, hash_alg, no_cutoff):
    P.test_decode_burst_alternate_key(dev, oracle_mod, hash_alg, no_cutoff)


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("hash_alg,enc_set,ivlen", [s for s in H.SETUPS if s[0]])
def test_host_bursts_wave_form(dev, virtual, oracle_mod, wave, k, hash_alg, enc_set,
                               ivlen):
    H.test_host_bursts_against_oracle(dev, virtual, oracle_mod, k, hash_alg, enc_set,
                                      ivlen)


def test_host_alternate_key_wave_form(dev, oracle_mod, wave):
    H.test_host_burst_alternate_key(dev, oracle_mod)


@pytest.mark.parametrize("gap", [0, 2000])
def test_host_pinned_layouts_wave_form(dev, oracle_mod, wave, gap):
    H.test_host_burst_pinned_layouts(dev, oracle_mod, gap)


@pytest.mark.parametrize("memory", ["pageable", "pinned"])
def test_host_large_datagrams_wave_form(dev, oracle_mod, wave, memory):
    H.test_host_burst_large_datagrams(dev, oracle_mod, memory)


def _burst(n, seed, hash_alg, enc_set):
    rng = np.random.default_rng(seed)
    hl = H.HL[hash_alg]
    want_flags = H.PH_SIGNED | (H.PH_ENCRYPTED if enc_set else 0)
    flags = np.full(n, want_flags, dtype=np.uint32)
    pick = rng.random(n)
    flags[pick < 0.08] ^= H.PH_SIGNED
    flags[(pick >= 0.08) & (pick < 0.16)] |= H.PH_ALTKEY
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    plen = rng.choice([0, 1, 55, 56, 111, 112, 119, 120, 127, 128, 500, 1428], n)
    slot = (8 + hl + plen).astype(np.uint32)
    short = rng.random(n) < 0.04                  # slots without room
    slot[short] = rng.integers(0, 8 + hl + 1, short.sum())
    import synth
    data, offs = synth.packed(seed + 1, slot, align=1, gap=5)
    return data, offs.astype(np.uint64), slot, seq, flags, rng


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 333, 1024, 2047, 5000, 16384, 16385])
@pytest.mark.parametrize("hash_alg,enc_set,ivlen", [(6, True, 16), (4, True, 32),
                                                    (5, False, 0)])
def test_small_host_bursts_default_threshold(dev, oracle_mod, n, hash_alg, enc_set,
                                             ivlen):
    """Integration-sized bursts at the default threshold (the wave form up
    to 16 datagrams per SIMD -- 1, 2, 5 and 16 datagrams per workgroup
    here -- the lane form above, unbinned below 65,536 datagrams): TX, then
    RX with tampered bytes and runts,
    pinned and pageable buffers, every code / sealed byte / header / IV
    against the oracle.  Message lengths straddle the padding boundaries
    (55/56, 111/112, 119/120 bytes: the length field in the tail block or a
    block of its own)."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    data, offs, slot, seq, flags, rng = _burst(n, 4000 + n + hash_alg, hash_alg,
                                                enc_set)
    key = rng.integers(0, 256, H.HL[hash_alg], dtype=np.uint8).tobytes()
    for memory in ("pageable", "pinned"):
        o_res, o_sealed = oracle_mod.packet_encode_batch(
            hash_alg, key, enc_set, seq, flags, data, offs, slot, nthreads=CPU_THREADS)
        if memory == "pinned":
            buf = H.pinned(data.shape, np.uint8)
            buf[:] = data
        else:
            buf = data.copy()
        res = H.encode_host(L, hash_alg, key, enc_set, seq, flags, buf, offs, slot)
        assert np.array_equal(res, o_res) and np.array_equal(buf, o_sealed), memory
        lens = slot.copy()
        t = rng.random(n)
        for i in np.nonzero((t < 0.1) & (lens > 8))[0]:
            buf[int(offs[i]) + 8 + int(rng.integers(0, lens[i] - 8))] ^= 0x10
        lens[(t >= 0.1) & (t < 0.13)] = 5
        want = oracle_mod.packet_decode_batch(hash_alg, key, enc_set, ivlen, buf, offs,
                                              lens, nthreads=CPU_THREADS)
        out = None
        if memory == "pinned":
            out = dict(res=H.pinned((n,), np.uint8),
                       iv=H.pinned((n, max(ivlen, 1)), np.uint8),
                       seq=H.pinned((n,), np.uint32), fl=H.pinned((n,), np.uint32))
            out["res"][:] = 9
        got = H.decode_host(L, H.rx_keys(hash_alg, key, enc_set), ivlen, buf, offs, lens,
                            out=out)
        H.check_decode(got, want, ivlen)


def test_wave_and_lane_forms_agree(dev, oracle_mod):
    """One device-resident burst of 1,000 datagrams decoded in both forms
    (net2_sha2_burst_limits wave_max 0: lane form; default: wave form): codes, decoded
    headers and the whole IV array -- rows left untouched included --
    identical, and equal to the oracle."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    n, hash_alg, ivlen = 1000, 6, 16
    data, offs, slot, seq, flags, rng = _burst(n, 4242, hash_alg, True)
    key = bytes(range(64))
    _, sealed = oracle_mod.packet_encode_batch(hash_alg, key, True, seq, flags, data,
                                               offs, slot, nthreads=CPU_THREADS)
    d = torch.from_numpy(sealed).to(dev)
    o = torch.from_numpy(offs.view(np.int64)).to(dev)
    ln = torch.from_numpy(slot.view(np.int32)).to(dev)
    ws = torch.empty(L.net2_packet_burst_workspace(n), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for wave_max in (0, -1):          # lane form, then the default (wave form)
        assert L.net2_sha2_burst_limits(wave_max, -1) == 0
        res = torch.full((n,), 9, dtype=torch.uint8, device=dev)
        iv = torch.full((n, ivlen), 0x5a, dtype=torch.uint8, device=dev)
        oseq = torch.full((n,), 7, dtype=torch.int32, device=dev)
        ofl = torch.full((n,), 7, dtype=torch.int32, device=dev)
        assert L.net2_packet_decode_burst(hash_alg, key, 64, 1, ivlen, d.data_ptr(),
                                          o.data_ptr(), ln.data_ptr(), n, res.data_ptr(),
                                          iv.data_ptr(), oseq.data_ptr(), ofl.data_ptr(),
                                          ws.data_ptr(), ws.numel(), st) == 0
        outs.append([x.cpu().numpy() for x in (res, iv, oseq, ofl)])
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    want = oracle_mod.packet_decode_batch(hash_alg, key, True, ivlen, sealed, offs, slot,
                                          nthreads=CPU_THREADS)
    assert np.array_equal(outs[1][0], want[0])
    assert (want[0] == 0).sum() > n // 2
