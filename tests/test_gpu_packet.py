"""Bursts of datagrams through the hash steps of net2_packet_encode / decode
(types/packet.n2t:341-463 / :170-336): net2_packet_encode_burst and
net2_packet_decode_burst against a line-by-line Python restatement of those
functions over the oracle's HMAC and net2_ph_to_iv (oracle/sha2_oracle.c).

Every burst mixes PH_SIGNED / PH_ENCRYPTED / other flag bits, runts shorter
than the header, signed datagrams too short for their hash field, tampered
payloads and hash fields, and flag / key mismatches (UNSAFE), under each
key set-up the negotiation can produce (keyed hash and cipher, either one,
neither).
"""
import ctypes
import errno
import os
import struct

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


def ref_decode(dg, hash_alg, key, enc_set, ivlen, oracle_mod):
    """net2_packet_decode (packet.n2t:170-336), hash steps only."""
    if len(dg) < 8:                                   # :196-198
        return BAD, None, None
    seq, fl = struct.unpack(">II", dg[:8])
    do_sign, do_cryp = fl & PH_SIGNED, fl & PH_ENCRYPTED
    if (not do_sign and hash_alg) or (not do_cryp and enc_set):   # :217-221
        return UNSAFE, (seq, fl), None
    rest = dg[8:]
    if do_sign:                                       # :226-258
        hl = HL[hash_alg]
        if len(rest) < hl:
            return BAD, (seq, fl), None
        supplied, msg = rest[:hl], rest[hl:]
        calc = oracle_mod.hmac(hash_alg, key, msg) if hash_alg else b""
        if supplied != calc:
            return BAD, (seq, fl), None
    iv = None
    if do_cryp and enc_set and ivlen:                 # :263-279
        iv = oracle_mod.ph_to_iv(seq, fl, ivlen)
    return OK, (seq, fl), iv


def ref_encode(slot, seq, fl, hash_alg, key, enc_set, oracle_mod):
    """net2_packet_encode (packet.n2t:341-463) on a slot laid out as header
    || reserved hash field (PH_SIGNED) || payload; returns (code, bytes)."""
    do_sign, do_cryp = fl & PH_SIGNED, fl & PH_ENCRYPTED
    if ((not do_sign and hash_alg) or (not do_cryp and enc_set) or
            (do_sign and not hash_alg) or (do_cryp and not enc_set)):  # :364-370
        return UNSAFE, slot
    hl = HL[hash_alg] if do_sign else 0
    if len(slot) < 8 + hl:
        return RESOURCE, slot
    payload = slot[8 + hl:]
    field = oracle_mod.hmac(hash_alg, key, payload) if do_sign else b""
    return OK, struct.pack(">II", seq, fl) + field + payload


def _dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


SETUPS = [(6, True, 16), (4, True, 16), (5, False, 0), (0, True, 32),
          (0, False, 0), (6, True, 64)]


@pytest.mark.parametrize("hash_alg,enc_set,ivlen", SETUPS)
def test_encode_then_decode_burst(dev, oracle_mod, hash_alg, enc_set, ivlen):
    from ilias_net2_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(1000 + 10 * hash_alg + ivlen + enc_set)
    n = 3001
    key = rng.integers(0, 256, HL[hash_alg], dtype=np.uint8).tobytes()
    want_flags = (PH_SIGNED if hash_alg else 0) | (PH_ENCRYPTED if enc_set else 0)
    # mostly the flags the keys call for; some wrong ones, some extra bits
    flags = np.full(n, want_flags, dtype=np.uint32)
    pick = rng.random(n)
    flags[pick < 0.1] ^= PH_SIGNED
    flags[(pick >= 0.1) & (pick < 0.2)] ^= PH_ENCRYPTED
    flags[(pick >= 0.2) & (pick < 0.3)] |= PH_ALTKEY | 0x10
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    plen = rng.choice([0, 1, 17, 64, 500, 1472], n)
    hl = np.where(flags & PH_SIGNED, HL[hash_alg], 0)
    slot = (8 + hl + plen).astype(np.uint32)
    short = rng.random(n) < 0.03              # slots with no room
    slot[short] = rng.integers(0, 8 + HL[hash_alg] + 1, short.sum())
    data, offs = synth.packed(1100 + hash_alg, slot, align=1, gap=3)
    kb = (key or b"\0")

    # ---- TX -------------------------------------------------------------
    d = _dev(data, dev)
    o, ln = _dev(offs.astype(np.int64), dev), _dev(slot.astype(np.int32), dev)
    ds, df = _dev(seq.view(np.int32), dev), _dev(flags.view(np.int32), dev)
    res = torch.full((n,), 9, dtype=torch.uint8, device=dev)
    ws = torch.empty(L.net2_packet_burst_workspace(n), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    rc = L.net2_packet_encode_burst(hash_alg, kb, len(key), int(enc_set), ds.data_ptr(),
                                    df.data_ptr(), d.data_ptr(), o.data_ptr(),
                                    ln.data_ptr(), n, res.data_ptr(), ws.data_ptr(),
                                    ws.numel(), st)
    assert rc == 0
    tx = d.cpu().numpy()
    got = res.cpu().numpy()
    for i in range(n):
        a, b = int(offs[i]), int(offs[i]) + int(slot[i])
        code, want = ref_encode(data[a:b].tobytes(), int(seq[i]), int(flags[i]),
                                hash_alg, key, enc_set, oracle_mod)
        assert got[i] == code, (i, got[i], code)
        assert tx[a:b].tobytes() == want, i

    # ---- RX: what TX produced, plus runts and tampered datagrams ---------
    rx = tx.copy()
    lens = slot.copy()
    tamper = rng.random(n)
    for i in range(n):
        a = int(offs[i])
        if tamper[i] < 0.05 and lens[i] > 8:       # flip a byte past the header
            j = a + 8 + int(rng.integers(0, lens[i] - 8))
            rx[j] ^= 0x40
        elif tamper[i] < 0.08:                     # runt
            lens[i] = int(rng.integers(0, 8))
    d2 = _dev(rx, dev)
    ln2 = _dev(lens.astype(np.int32), dev)
    res.fill_(9)
    iv = torch.zeros((n, max(ivlen, 1)), dtype=torch.uint8, device=dev)
    oseq = torch.zeros(n, dtype=torch.int32, device=dev)
    ofl = torch.zeros(n, dtype=torch.int32, device=dev)
    rc = L.net2_packet_decode_burst(hash_alg, kb, len(key), int(enc_set), ivlen,
                                    d2.data_ptr(), o.data_ptr(), ln2.data_ptr(), n,
                                    res.data_ptr(), iv.data_ptr() if ivlen else None,
                                    oseq.data_ptr(), ofl.data_ptr(), ws.data_ptr(),
                                    ws.numel(), st)
    assert rc == 0
    got = res.cpu().numpy()
    giv = iv.cpu().numpy()
    gseq = oseq.cpu().numpy().view(np.uint32)
    gfl = ofl.cpu().numpy().view(np.uint32)
    counts = {}
    for i in range(n):
        a = int(offs[i])
        dg = rx[a:a + int(lens[i])].tobytes()
        code, hdr, want_iv = ref_decode(dg, hash_alg, key, enc_set, ivlen, oracle_mod)
        counts[code] = counts.get(code, 0) + 1
        assert got[i] == code, (i, got[i], code)
        if hdr is not None:
            assert (gseq[i], gfl[i]) == hdr, i
        if want_iv is not None:
            assert giv[i, :ivlen].tobytes() == want_iv, i
    # every outcome the set-up allows actually occurred
    assert counts.get(OK, 0) > n // 2 and counts.get(BAD, 0) > 0
    if hash_alg or enc_set:
        assert counts.get(UNSAFE, 0) > 0


def test_burst_argument_errors(dev):
    from ilias_net2_amd import _lib
    import errno
    L = _lib.lib()
    t = torch.zeros(256, dtype=torch.uint8, device=dev)
    p = t.data_ptr()
    ws = L.net2_packet_burst_workspace(4)
    w = torch.zeros(ws, dtype=torch.uint8, device=dev)
    key = b"k" * 64
    # unkeyed row, wrong key length, ivlen > 64, workspace too small
    assert L.net2_packet_decode_burst(1, key, 0, 0, 0, p, p, p, 4, p, None, None,
                                      None, w.data_ptr(), ws, None) == errno.EINVAL
    assert L.net2_packet_decode_burst(4, key, 31, 0, 0, p, p, p, 4, p, None, None,
                                      None, w.data_ptr(), ws, None) == errno.EINVAL
    assert L.net2_packet_decode_burst(0, None, 0, 1, 65, p, p, p, 4, p, p, None,
                                      None, w.data_ptr(), ws, None) == errno.EINVAL
    assert L.net2_packet_decode_burst(0, None, 0, 0, 0, p, p, p, 4, p, None, None,
                                      None, w.data_ptr(), ws - 1, None) == errno.EINVAL
    assert L.net2_packet_encode_burst(4, key, 32, 0, None, None, p, p, p, 4, p,
                                      w.data_ptr(), ws, None) == errno.EINVAL
    # an empty burst is a no-op
    assert L.net2_packet_decode_burst(0, None, 0, 0, 0, None, None, None, 0, None,
                                      None, None, None, None, 0, None) == 0


def ref_rx_key(seq, fl, has_alt, no_cutoff, cutoff, rx_start):
    """net2_ck_rx_key (src/conn_keys.c:447-476): True for the alternate
    key.  u32 wrap-around as in C."""
    if not has_alt:
        return False
    return bool(fl & PH_ALTKEY) or (
        not no_cutoff and ((seq - rx_start) & 0xffffffff) >=
        ((cutoff - rx_start) & 0xffffffff))


@pytest.mark.parametrize("hash_alg,no_cutoff", [(6, False), (6, True), (4, False), (5, False)])
def test_decode_burst_alternate_key(dev, oracle_mod, hash_alg, no_cutoff):
    """A burst received during a key rollover: each datagram sealed with the
    key net2_ck_rx_key picks for its header (PH_ALTKEY, or a seq past the
    cutoff, the window start wrapping around), plus datagrams sealed with
    the other key -- those must come out NET2_PDECODE_BAD, as the
    reference's hash compare makes them (packet.n2t:226-258)."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(7000 + hash_alg + 10 * no_cutoff)
    n, hl, ivlen = 2500, HL[hash_alg], 16
    key = rng.integers(0, 256, hl, dtype=np.uint8).tobytes()
    alt = rng.integers(0, 256, hl, dtype=np.uint8).tobytes()
    rx_start = 0xfffff000                     # the window start wraps
    cutoff = (rx_start + 1200) & 0xffffffff
    seq = ((rx_start + rng.integers(0, 2500, n)) & 0xffffffff).astype(np.uint32)
    flags = np.full(n, PH_SIGNED | PH_ENCRYPTED, dtype=np.uint32)
    flags[rng.random(n) < 0.3] |= PH_ALTKEY
    wrong = rng.random(n) < 0.1               # sealed with the other key
    plen = rng.choice([0, 5, 64, 300, 1400], n)
    dgs, want = [], []
    for i in range(n):
        use_alt = ref_rx_key(int(seq[i]), int(flags[i]), True, no_cutoff, cutoff, rx_start)
        k = (alt if use_alt else key) if not wrong[i] else (key if use_alt else alt)
        payload = rng.integers(0, 256, int(plen[i]), dtype=np.uint8).tobytes()
        dgs.append(struct.pack(">II", int(seq[i]), int(flags[i])) +
                   oracle_mod.hmac(hash_alg, k, payload) + payload)
        want.append(BAD if wrong[i] else OK)
    lens = np.array([len(d) for d in dgs], dtype=np.uint32)
    data, offs = synth.packed(9000 + hash_alg, lens, align=1)
    for i, d in enumerate(dgs):
        data[int(offs[i]):int(offs[i]) + len(d)] = np.frombuffer(d, dtype=np.uint8)
    d = _dev(data, dev)
    o, ln = _dev(offs.astype(np.int64), dev), _dev(lens.astype(np.int32), dev)
    res = torch.full((n,), 9, dtype=torch.uint8, device=dev)
    iv = torch.zeros((n, ivlen), dtype=torch.uint8, device=dev)
    ws = torch.empty(L.net2_packet_burst_workspace(n), dtype=torch.uint8, device=dev)
    kb, ab = ctypes.create_string_buffer(key, hl), ctypes.create_string_buffer(alt, hl)
    ks = _lib.BurstRxKeys(hash_alg, ctypes.cast(kb, ctypes.c_void_p), hl, 1,
                          ctypes.cast(ab, ctypes.c_void_p), hl, int(no_cutoff),
                          cutoff, rx_start)
    st = torch.cuda.current_stream().cuda_stream
    rc = L.net2_packet_decode_burst_ck(ctypes.byref(ks), ivlen, d.data_ptr(),
                                       o.data_ptr(), ln.data_ptr(), n, res.data_ptr(),
                                       iv.data_ptr(), None, None, ws.data_ptr(),
                                       ws.numel(), st)
    assert rc == 0
    got = res.cpu().numpy()
    giv = iv.cpu().numpy()
    assert list(got) == want
    for i in np.nonzero(got == OK)[0][:200]:
        assert giv[i].tobytes() == oracle_mod.ph_to_iv(int(seq[i]), int(flags[i]), ivlen)
    # both keys were used, and the plain entry point (no alternate key)
    # accepts exactly the datagrams sealed with the active key
    picks = [ref_rx_key(int(seq[i]), int(flags[i]), True, no_cutoff, cutoff, rx_start)
             for i in range(n)]
    assert 0 < sum(picks) < n
    res.fill_(9)
    rc = L.net2_packet_decode_burst(hash_alg, kb, hl, 1, ivlen, d.data_ptr(),
                                    o.data_ptr(), ln.data_ptr(), n, res.data_ptr(),
                                    None, None, None, ws.data_ptr(), ws.numel(), st)
    assert rc == 0
    sealed_active = [(not p) != bool(w) for p, w in zip(picks, wrong)]
    assert list(res.cpu().numpy()) == [OK if s else BAD for s in sealed_active]
    # the alternate key's length must match the active key's
    ks.alt_hash_keylen = hl - 1
    assert L.net2_packet_decode_burst_ck(ctypes.byref(ks), ivlen, d.data_ptr(),
                                         o.data_ptr(), ln.data_ptr(), n, res.data_ptr(),
                                         iv.data_ptr(), None, None, ws.data_ptr(),
                                         ws.numel(), st) == errno.EINVAL


def test_burst_round_trip_full_size(dev, oracle_mod):
    """The burst bench config at full size (1 M wire datagrams of {136, 584,
    1500} B, HMAC-SHA512, 16-byte IVs), every result against the oracle's
    restatement of the packet.n2t hash steps (oracle_packet_encode_batch /
    _decode_batch): the sealed bytes and codes of every slot, then the
    decode codes, headers and IVs of every datagram, intact and with one
    payload byte flipped in a chosen set.  Kept beside them, the
    size-independent properties: encode then decode accepts everything, the
    IVs equal net2_ph_to_iv_dev's, exactly the tampered datagrams fail."""
    from ilias_net2_amd import _lib
    L = _lib.lib()
    n, hl, ivlen, alg = 1 << 20, 64, 16, 6
    g = torch.Generator(device=dev)
    g.manual_seed(41)
    choice = torch.tensor([136, 584, 1500], dtype=torch.int64, device=dev)
    lens = choice[torch.randint(0, 3, (n,), device=dev, generator=g)]
    offs = torch.zeros(n, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)[:-1]
    data = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8,
                         device=dev, generator=g)
    l32 = lens.to(torch.int32)
    seq = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev,
                        generator=g)
    flags = torch.full((n,), PH_SIGNED | PH_ENCRYPTED, dtype=torch.int32, device=dev)
    key = bytes(range(7, 7 + hl))
    offs_h, lens_h = offs.cpu().numpy(), lens.cpu().numpy()
    seq_h = seq.cpu().numpy().view(np.uint32)
    fl_h = flags.cpu().numpy().view(np.uint32)
    o_res, o_sealed = oracle_mod.packet_encode_batch(
        alg, key, True, seq_h, fl_h, data.cpu().numpy(), offs_h, lens_h,
        nthreads=CPU_THREADS)
    res = torch.full((n,), 9, dtype=torch.uint8, device=dev)
    ws = torch.empty(L.net2_packet_burst_workspace(n), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    assert L.net2_packet_encode_burst(alg, key, hl, 1, seq.data_ptr(), flags.data_ptr(),
                                      data.data_ptr(), offs.data_ptr(), l32.data_ptr(),
                                      n, res.data_ptr(), ws.data_ptr(), ws.numel(), st) == 0
    assert int((res != OK).sum()) == 0
    assert np.array_equal(res.cpu().numpy(), o_res)
    assert np.array_equal(data.cpu().numpy(), o_sealed)  # every sealed byte
    del o_sealed

    def decode(buf):
        res.fill_(9)
        iv = torch.zeros((n, ivlen), dtype=torch.uint8, device=dev)
        oseq = torch.zeros(n, dtype=torch.int32, device=dev)
        ofl = torch.zeros(n, dtype=torch.int32, device=dev)
        assert L.net2_packet_decode_burst(alg, key, hl, 1, ivlen, buf.data_ptr(),
                                          offs.data_ptr(), l32.data_ptr(), n,
                                          res.data_ptr(), iv.data_ptr(), oseq.data_ptr(),
                                          ofl.data_ptr(), ws.data_ptr(), ws.numel(),
                                          st) == 0
        return res.clone(), iv, oseq, ofl

    def against_oracle(buf, got, iv, oseq, ofl):
        o_res, o_iv, o_seq, o_fl = oracle_mod.packet_decode_batch(
            alg, key, True, ivlen, buf.cpu().numpy(), offs_h, lens_h,
            nthreads=CPU_THREADS)
        assert np.array_equal(got.cpu().numpy(), o_res)
        assert np.array_equal(oseq.cpu().numpy().view(np.uint32), o_seq)
        assert np.array_equal(ofl.cpu().numpy().view(np.uint32), o_fl)
        ok = o_res == OK
        assert np.array_equal(iv.cpu().numpy()[ok], o_iv[ok])
        return o_res

    got, iv, oseq, ofl = decode(data)
    assert int((got != OK).sum()) == 0
    against_oracle(data, got, iv, oseq, ofl)
    assert torch.equal(oseq, seq) and torch.equal(ofl, flags)
    want_iv = torch.empty_like(iv)
    assert L.net2_ph_to_iv_dev(seq.data_ptr(), flags.data_ptr(), n, ivlen,
                               want_iv.data_ptr(), st) == 0
    assert torch.equal(iv, want_iv)
    # and the IVs of every header through the oracle's ph_to_iv batch
    assert np.array_equal(iv.cpu().numpy(), oracle_mod.ph_to_iv_batch(
        seq_h, fl_h, ivlen, nthreads=CPU_THREADS))
    # tamper with a chosen set: exactly those fail the hash compare
    rng = np.random.default_rng(42)
    bad = np.sort(rng.choice(n, 4096, replace=False))
    pos = offs_h[bad] + 8 + rng.integers(0, lens_h[bad] - 8)
    t = data.clone()
    idx = torch.from_numpy(pos.astype(np.int64)).to(dev)
    t[idx] ^= 0x20
    got, iv, oseq, ofl = decode(t)
    o_res = against_oracle(t, got, iv, oseq, ofl)
    assert np.array_equal(np.nonzero(o_res)[0], bad)
    want = torch.zeros(n, dtype=torch.uint8, device=dev)
    want[torch.from_numpy(bad.astype(np.int64)).to(dev)] = BAD
    assert torch.equal(got, want)
