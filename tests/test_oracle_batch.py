"""The oracle's threaded batch forms (oracle/sha2_oracle.c: HMAC,
net2_ph_to_iv, the hash steps of net2_packet_decode / _encode) pinned on
the CPU before the full-size GPU tests use them as the checker of every
result: against Python's hmac / hashlib (independent implementations), RFC
4231 through the batch entry point, the oracle's own one-item functions,
and a line-by-line Python restatement of types/packet.n2t:170-336 /
:341-463 (the same restatement tests/test_gpu_packet.py checks the GPU
bursts against).  CPU only."""
import hashlib
import hmac as pyhmac
import struct

import numpy as np

import synth

PH_ENCRYPTED, PH_SIGNED, PH_ALTKEY = 0x1, 0x2, 0x80000000
OK, RESOURCE, BAD, UNSAFE = 0, 1, 2, 3
HL = {0: 0, 4: 32, 5: 48, 6: 64}
HN = {4: "sha256", 5: "sha384", 6: "sha512"}


def _py_hmac(alg, key, m):
    return pyhmac.new(key, m, HN[alg]).digest()


def test_hmac_batch_layouts_vs_python(oracle_mod):
    for alg in (4, 5, 6):
        for keylen in (0, 4, 32, 64, 129, 200):
            key = bytes(synth.random_bytes(300 + keylen, keylen))
            lens = np.array([0, 1, 55, 56, 63, 64, 111, 112, 127, 128, 129,
                             500, 1500, 4097], dtype=np.uint32)
            data, offs = synth.packed(400 + alg, lens, align=1, gap=3)
            got = oracle_mod.hmac_batch(alg, key, data, offsets=offs, lens=lens,
                                        nthreads=3)
            for i in range(len(lens)):
                m = data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
                assert got[i].tobytes() == _py_hmac(alg, key, m), (alg, keylen, i)
        fixed = synth.fixed_batch(500 + alg, 97, 700, 704)
        got = oracle_mod.hmac_batch(alg, b"k" * 20, fixed, stride=704, length=700,
                                    n=97, nthreads=4)
        for i in range(97):
            m = fixed[i * 704:i * 704 + 700].tobytes()
            assert got[i].tobytes() == _py_hmac(alg, b"k" * 20, m)


def test_hmac_batch_rfc4231(oracle_mod, golden):
    for c in golden["kat"]["rfc4231"]:
        key, data = bytes.fromhex(c["key"]), bytes.fromhex(c["data"])
        arr = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, np.uint8)
        for alg, name in ((4, "HMAC-SHA256"), (5, "HMAC-SHA384"), (6, "HMAC-SHA512")):
            got = oracle_mod.hmac_batch(alg, key, arr, offsets=[0], lens=[len(data)])
            assert got[0].tobytes().hex()[:len(c[name])] == c[name]


def test_ph_to_iv_batch(oracle_mod):
    rng = np.random.default_rng(5)
    seq = rng.integers(0, 2**32, 500, dtype=np.uint64).astype(np.uint32)
    fl = rng.integers(0, 2**32, 500, dtype=np.uint64).astype(np.uint32)
    for ivlen in (1, 16, 32, 33, 64, 100):
        got = oracle_mod.ph_to_iv_batch(seq, fl, ivlen, nthreads=4)
        for i in range(0, 500, 7):
            ph = struct.pack(">II", int(seq[i]), int(fl[i]))
            iv = b""
            while len(iv) < ivlen:                     # packet.n2t:127-144
                iv += hashlib.sha256(ph + iv).digest()[:ivlen - len(iv)]
            assert got[i].tobytes() == iv
            assert oracle_mod.ph_to_iv(int(seq[i]), int(fl[i]), ivlen) == iv


def _ref_rx_key(seq, fl, alt, no_cutoff, cutoff, rx_start):
    """net2_ck_rx_key (src/conn_keys.c:447-476)."""
    return alt is not None and (bool(fl & PH_ALTKEY) or (
        not no_cutoff and ((seq - rx_start) & 0xffffffff) >=
        ((cutoff - rx_start) & 0xffffffff)))


def _ref_decode(dg, hash_alg, key, enc_set, ivlen, alt=None, no_cutoff=False,
                cutoff=0, rx_start=0):
    """net2_packet_decode (packet.n2t:170-336), hash steps only, with
    Python's hmac / hashlib."""
    if len(dg) < 8:                                     # :196-198
        return BAD, None, None
    seq, fl = struct.unpack(">II", dg[:8])
    if _ref_rx_key(seq, fl, alt, no_cutoff, cutoff, rx_start):   # :210
        key = alt
    if (not fl & PH_SIGNED and hash_alg) or (not fl & PH_ENCRYPTED and enc_set):
        return UNSAFE, (seq, fl), None                  # :217-221
    rest = dg[8:]
    if fl & PH_SIGNED:                                  # :226-258
        hl = HL[hash_alg]
        if len(rest) < hl:
            return BAD, (seq, fl), None
        if hl and rest[:hl] != _py_hmac(hash_alg, key, rest[hl:]):
            return BAD, (seq, fl), None
    iv = None
    if fl & PH_ENCRYPTED and enc_set and ivlen:         # :263-279
        ph, iv = dg[:8], b""
        while len(iv) < ivlen:
            iv += hashlib.sha256(ph + iv).digest()[:ivlen - len(iv)]
    return OK, (seq, fl), iv


def _burst(seed, hash_alg, enc_set, n=1500):
    rng = np.random.default_rng(seed)
    hl = HL[hash_alg]
    key = rng.integers(0, 256, hl, dtype=np.uint8).tobytes()
    want_flags = (PH_SIGNED if hash_alg else 0) | (PH_ENCRYPTED if enc_set else 0)
    flags = np.full(n, want_flags, dtype=np.uint32)
    pick = rng.random(n)
    flags[pick < 0.1] ^= PH_SIGNED
    flags[(pick >= 0.1) & (pick < 0.2)] ^= PH_ENCRYPTED
    flags[(pick >= 0.2) & (pick < 0.4)] |= PH_ALTKEY | 0x10
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    plen = rng.choice([0, 1, 17, 64, 500, 1472], n)
    slot = (8 + np.where(flags & PH_SIGNED, hl, 0) + plen).astype(np.uint32)
    short = rng.random(n) < 0.03
    slot[short] = rng.integers(0, 8 + hl + 1, short.sum())
    data, offs = synth.packed(seed + 1, slot, align=1, gap=3)
    return rng, key, flags, seq, slot, data, offs


def _ref_encode(slot, seq, fl, hash_alg, key, enc_set):
    """net2_packet_encode (packet.n2t:341-463) hash steps."""
    do_sign, do_cryp = fl & PH_SIGNED, fl & PH_ENCRYPTED
    if ((not do_sign and hash_alg) or (not do_cryp and enc_set) or
            (do_sign and not hash_alg) or (do_cryp and not enc_set)):
        return UNSAFE, slot
    hl = HL[hash_alg] if do_sign else 0
    if len(slot) < 8 + hl:
        return RESOURCE, slot
    payload = slot[8 + hl:]
    field = _py_hmac(hash_alg, key, payload) if do_sign else b""
    return OK, struct.pack(">II", seq, fl) + field + payload


def test_packet_encode_decode_batch_vs_restatement(oracle_mod):
    for hash_alg, enc_set, ivlen in [(6, True, 16), (4, True, 16), (5, False, 0),
                                     (0, True, 32), (0, False, 0), (6, True, 64)]:
        rng, key, flags, seq, slot, data, offs = _burst(
            2000 + hash_alg + ivlen, hash_alg, enc_set)
        n = len(slot)
        res, sealed = oracle_mod.packet_encode_batch(hash_alg, key, enc_set, seq,
                                                     flags, data, offs, slot,
                                                     nthreads=4)
        for i in range(n):
            a, b = int(offs[i]), int(offs[i]) + int(slot[i])
            code, want = _ref_encode(data[a:b].tobytes(), int(seq[i]),
                                     int(flags[i]), hash_alg, key, enc_set)
            assert res[i] == code, (i, res[i], code)
            assert sealed[a:b].tobytes() == want, i
        rx, lens = sealed.copy(), slot.copy()
        for i in range(n):
            a = int(offs[i])
            t = rng.random()
            if t < 0.05 and lens[i] > 8:
                rx[a + 8 + int(rng.integers(0, lens[i] - 8))] ^= 0x40
            elif t < 0.08:
                lens[i] = int(rng.integers(0, 8))
        res, iv, s_out, f_out = oracle_mod.packet_decode_batch(
            hash_alg, key, enc_set, ivlen, rx, offs, lens, nthreads=4)
        seen = set()
        for i in range(n):
            a = int(offs[i])
            code, hdr, want_iv = _ref_decode(rx[a:a + int(lens[i])].tobytes(),
                                             hash_alg, key, enc_set, ivlen)
            seen.add(code)
            assert res[i] == code, (i, res[i], code)
            if hdr is not None:
                assert (int(s_out[i]), int(f_out[i])) == hdr
            if want_iv is not None:
                assert iv[i].tobytes() == want_iv
            elif ivlen:
                assert not iv[i].any()
        assert OK in seen and BAD in seen


def test_packet_decode_batch_alternate_key(oracle_mod):
    rng = np.random.default_rng(77)
    n, alg, hl = 800, 6, 64
    key = rng.integers(0, 256, hl, dtype=np.uint8).tobytes()
    alt = rng.integers(0, 256, hl, dtype=np.uint8).tobytes()
    rx_start = 0xfffff000
    cutoff = (rx_start + 400) & 0xffffffff
    for no_cutoff in (False, True):
        seq = ((rx_start + rng.integers(0, 800, n)) & 0xffffffff).astype(np.uint32)
        fl = np.full(n, PH_SIGNED | PH_ENCRYPTED, dtype=np.uint32)
        fl[rng.random(n) < 0.3] |= PH_ALTKEY
        dgs = []
        for i in range(n):
            use_alt = _ref_rx_key(int(seq[i]), int(fl[i]), alt, no_cutoff, cutoff, rx_start)
            k = alt if (use_alt != (i % 9 == 0)) else key   # every 9th: wrong key
            p = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
            dgs.append(struct.pack(">II", int(seq[i]), int(fl[i])) + _py_hmac(alg, k, p) + p)
        lens = np.array([len(d) for d in dgs], dtype=np.uint32)
        data, offs = synth.packed(78, lens)
        for i, d in enumerate(dgs):
            data[int(offs[i]):int(offs[i]) + len(d)] = np.frombuffer(d, np.uint8)
        res, iv, _, _ = oracle_mod.packet_decode_batch(
            alg, key, True, 16, data, offs, lens, alt_key=alt,
            alt_no_cutoff=no_cutoff, alt_cutoff=cutoff, rx_start=rx_start)
        for i in range(n):
            code, _, want_iv = _ref_decode(dgs[i], alg, key, True, 16, alt,
                                           no_cutoff, cutoff, rx_start)
            assert res[i] == code and code == (BAD if i % 9 == 0 else OK), i
            if want_iv is not None:
                assert iv[i].tobytes() == want_iv
