"""CPU: the oracle is pinned before anything is checked against it.

Pins: the reference's own KATs (test/hash.cc:21-48), FIPS 180-4 examples, the
RFC 4231 HMAC test cases (published MACs), and Python hashlib / hmac as
independent implementations.  tests/golden/survey_ref_sha2c.json holds outputs
of a survey-time build of src/sha2.c with a reconstructed header -- a
cross-check, not a reference pin (the header is a stand-in).  Also the
SHA2_CTX call semantics of src/sha2.c that callers can observe.
"""
import ctypes
import hashlib
import hmac as pyhmac

import numpy as np
import pytest

import synth
from golden.make_golden import FIPS_MESSAGES, pattern

NAMES = {1: "SHA256", 2: "SHA384", 3: "SHA512"}
HL = {1: hashlib.sha256, 2: hashlib.sha384, 3: hashlib.sha512}


def test_reference_kat(oracle_mod, golden):
    ref = golden["kat"]["reference"]
    msg = ref["message"].encode()
    for alg, name in NAMES.items():
        assert oracle_mod.digest(alg, msg).hex() == ref[name]
    assert ref["SHA256"].startswith("5d8082c2")  # test/hash.cc:24


def test_survey_build_outputs(oracle_mod, golden):
    """Survey-time build of src/sha2.c with a reconstructed sha2.h (SURVEY.md
    8c): agreement is a cross-check only, not a pin."""
    for n, v in golden["sha2c"]["vectors"].items():
        m = pattern(int(n))
        assert oracle_mod.digest(1, m).hex() == v["SHA256"]
        assert oracle_mod.digest(3, m).hex().startswith(v["SHA512_prefix"])


@pytest.mark.parametrize("key", sorted(FIPS_MESSAGES))
def test_fips(oracle_mod, golden, key):
    for alg, name in NAMES.items():
        assert oracle_mod.digest(alg, FIPS_MESSAGES[key]).hex() == golden["kat"]["fips"][key][name]


def test_fips_abc_published():
    # FIPS 180-4 appendix values, independent of every implementation here
    from oracle import oracle
    assert oracle.digest(1, b"abc").hex() == (
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad")
    assert oracle.digest(3, b"abc").hex().startswith("ddaf35a193617aba")


def test_boundaries(oracle_mod, golden):
    for n, row in golden["kat"]["boundary"].items():
        m = pattern(int(n))
        for alg, name in NAMES.items():
            assert oracle_mod.digest(alg, m).hex() == row[name], (n, name)


def test_random_vs_hashlib(oracle_mod):
    rng = np.random.default_rng(11)
    for n in list(range(0, 260)) + [1499, 1500, 1501, 8191]:
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for alg in NAMES:
            assert oracle_mod.digest(alg, m) == HL[alg](m).digest()


def test_hmac(oracle_mod, golden):
    for v in golden["kat"]["hmac"]:
        key = bytes.fromhex(v["key"])
        m = pattern(v["len"])
        assert oracle_mod.hmac(v["alg"], key, m).hex() == v["digest"]
        h = {4: "sha256", 5: "sha384", 6: "sha512"}[v["alg"]]
        assert pyhmac.new(key, m, h).hexdigest() == v["digest"]


def test_rfc4231(oracle_mod, golden):
    """RFC 4231 section 4, cases 1-7: keys of 4, 20, 25 and 131 bytes (the
    last hashed first), data shorter and longer than a block; case 5 is
    compared on the 128 bits the RFC publishes."""
    cases = golden["kat"]["rfc4231"]
    assert [c["case"] for c in cases] == list(range(1, 8))
    assert cases[0]["HMAC-SHA256"].startswith("b0344c61")  # RFC 4231 4.2
    for c in cases:
        key, data = bytes.fromhex(c["key"]), bytes.fromhex(c["data"])
        for alg, name in ((4, "HMAC-SHA256"), (5, "HMAC-SHA384"),
                          (6, "HMAC-SHA512")):
            want = c[name]
            assert oracle_mod.hmac(alg, key, data).hex()[:len(want)] == want, (c["case"], name)


def test_batches(oracle_mod, golden):
    for b in golden["batches"]:
        if b["kind"] == "fixed":
            data = synth.fixed_batch(b["seed"], b["n"], b["len"], b["stride"])
            d = oracle_mod.batch(b["alg"], data, stride=b["stride"],
                                 length=b["len"], n=b["n"], nthreads=4)
        else:
            lens = synth.mixed_lengths(b["len_seed"], b["n"])
            data, offs = synth.packed(b["seed"], lens, align=b["align"])
            d = oracle_mod.batch(b["alg"], data, offsets=offs, lens=lens,
                                 nthreads=3)
        assert hashlib.sha256(d.tobytes()).hexdigest() == b["digest_of_digests"]
        assert d[0].tobytes().hex() == b["first"]
        assert d[-1].tobytes().hex() == b["last"]


def test_unrolled_variant(oracle_mod, golden):
    """The SHA2_UNROLL_TRANSFORM form (src/sha2.c:316-370, :605-659) that the
    CPU baseline also times: same digests as the rolled form on the golden
    batches and on every padding boundary 0..300 bytes."""
    for b in golden["batches"]:
        if b["kind"] == "fixed":
            data = synth.fixed_batch(b["seed"], b["n"], b["len"], b["stride"])
            d = oracle_mod.batch(b["alg"], data, stride=b["stride"],
                                 length=b["len"], n=b["n"], nthreads=2,
                                 unrolled=True)
        else:
            lens = synth.mixed_lengths(b["len_seed"], b["n"])
            data, offs = synth.packed(b["seed"], lens, align=b["align"])
            d = oracle_mod.batch(b["alg"], data, offsets=offs, lens=lens,
                                 nthreads=2, unrolled=True)
        assert hashlib.sha256(d.tobytes()).hexdigest() == b["digest_of_digests"]
    lens = np.arange(301, dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = synth.random_bytes(9, int(lens.sum()))
    for alg, h in ((1, hashlib.sha256), (2, hashlib.sha384), (3, hashlib.sha512)):
        d = oracle_mod.batch(alg, data, offsets=offs, lens=lens, unrolled=True)
        for i in range(len(lens)):
            m = bytes(data[int(offs[i]):int(offs[i]) + int(lens[i])])
            assert d[i].tobytes() == h(m).digest(), (alg, i)


def test_openssl_context_baseline(oracle_mod, golden):
    """The OpenSSL leg of bench.py's cpu_baseline (oracle/openssl_batch.c,
    SHA*_Init/Update/Final as cxx_src/hash-openssl.cc calls them) hashes
    the golden batches to the same digests."""
    for b in golden["batches"]:
        if b["kind"] == "fixed":
            data = synth.fixed_batch(b["seed"], b["n"], b["len"], b["stride"])
            d = oracle_mod.openssl_batch(b["alg"], data, stride=b["stride"],
                                         length=b["len"], n=b["n"], nthreads=3)
        else:
            lens = synth.mixed_lengths(b["len_seed"], b["n"])
            data, offs = synth.packed(b["seed"], lens, align=b["align"])
            d = oracle_mod.openssl_batch(b["alg"], data, offsets=offs,
                                         lens=lens, nthreads=2)
        assert hashlib.sha256(d.tobytes()).hexdigest() == b["digest_of_digests"]


def _ctx_digest(L, pfx, chunks, dl):
    ctx = ctypes.create_string_buffer(208)
    getattr(L, f"oracle_{pfx}_init")(ctx)
    for c in chunks:
        buf = ctypes.create_string_buffer(c, max(len(c), 1))
        getattr(L, f"oracle_{pfx}_update")(ctx, buf, len(c))
    out = ctypes.create_string_buffer(64)
    getattr(L, f"oracle_{pfx}_final")(out, ctx)
    return out.raw[:dl], ctx.raw


def test_streaming_semantics(oracle_mod):
    """Init/Update/Final over arbitrary split points == one shot
    (src/sha2.c:449-493 buffering); Update(len 0) is a no-op (:455)."""
    L = oracle_mod.lib()
    rng = np.random.default_rng(5)
    for pfx, alg, dl in (("sha256", 1, 32), ("sha384", 2, 48), ("sha512", 3, 64)):
        for n in (0, 1, 63, 64, 65, 127, 128, 129, 1000):
            m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            cuts = sorted(rng.integers(0, n + 1, 4).tolist())
            chunks = [m[a:b] for a, b in zip([0] + cuts, cuts + [n])]
            chunks.insert(1, b"")
            d, ctx_after = _ctx_digest(L, pfx, chunks, dl)
            assert d == HL[alg](m).digest()
            assert ctx_after == b"\0" * 208  # zeroed after a real Final


def test_final_null_keeps_state(oracle_mod):
    """Final(NULL) pads but keeps the ctx for SHA-256/512 (src/sha2.c:551-562,
    840-858); SHA-384 zeroes it regardless (src/sha2.c:918)."""
    L = oracle_mod.lib()
    for pfx, zeroed in (("sha256", False), ("sha512", False), ("sha384", True)):
        ctx = ctypes.create_string_buffer(208)
        getattr(L, f"oracle_{pfx}_init")(ctx)
        getattr(L, f"oracle_{pfx}_update")(ctx, b"abc", 3)
        getattr(L, f"oracle_{pfx}_final")(None, ctx)
        assert (ctx.raw == b"\0" * 208) == zeroed, pfx


def test_init_null_is_noop(oracle_mod):
    L = oracle_mod.lib()
    for pfx in ("sha256", "sha384", "sha512"):
        getattr(L, f"oracle_{pfx}_init")(None)  # must not crash (src/sha2.c:283)
