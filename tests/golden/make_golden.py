"""Regenerate the golden vectors under tests/golden/.

Sources, in order of authority:
  1. the reference's own known-answer tests, test/hash.cc:21-48 (SHA-256/384/
     512 of "Luke, I am your father."), copied here as data;
  2. FIPS 180-4 / NIST CAVP example messages ("abc", "", the 448- and 896-bit
     messages, one million 'a');
  3. boundary-length and seeded-batch vectors produced by the CPU oracle
     (oracle/sha2_oracle.c), each cross-checked against Python hashlib before
     it is written -- the script refuses to write a vector they disagree on.

The reference's src/sha2.c cannot be compiled in this image (it includes the
absent include/ilias/net2/bsd_compat/sha2.h), so no vector comes from it
directly; see DESIGN.md "Oracle".

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import hmac as pyhmac
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle  # noqa: E402
import synth  # noqa: E402

ALGS = {1: ("SHA256", hashlib.sha256), 2: ("SHA384", hashlib.sha384),
        3: ("SHA512", hashlib.sha512)}

# test/hash.cc:23-48, verbatim digests (data, not code)
REFERENCE_KAT = {
    "message": "Luke, I am your father.",
    "SHA256": "5d8082c2eabfe36a513a644700155bc479ceee8533459e71678b689beabdd7d6",
    "SHA384": ("ec2c17ed886aa29b3067690de319cfdcad69313e00390339d56dfec13dde384b"
               "f06342cdf9f58ffb5a9fcdfcc9db3c93"),
    "SHA512": ("9759a18565f81720c112d84041ec1aa23196378d27cfe0f47ad35d0afad58421"
               "3846f46f50994168ed0993be1193dc592b1a04f0404b9df587175974c97a1ffe"),
    "source": "test/hash.cc:21-48",
}

FIPS_MESSAGES = {
    "empty": b"",
    "abc": b"abc",
    "448bit": b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
    "896bit": (b"abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmn"
               b"hijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu"),
    "million_a": b"a" * 1_000_000,
}

BOUNDARY_LENGTHS = [0, 1, 3, 4, 5, 31, 32, 55, 56, 57, 63, 64, 65, 111, 112,
                    113, 119, 120, 127, 128, 129, 191, 192, 255, 256, 1000,
                    1023, 1024, 1025, 1500, 4096, 65535, 65536]


def pattern(n: int) -> bytes:
    """m[i] = (7 i + 3) mod 256."""
    return bytes(((7 * i + 3) & 0xFF) for i in range(n))


def checked(alg: int, msg: bytes) -> str:
    d = oracle.digest(alg, msg)
    if d != ALGS[alg][1](msg).digest():
        raise SystemExit(f"oracle/hashlib disagree: alg {alg} len {len(msg)}")
    return d.hex()


def make_kat():
    msg = REFERENCE_KAT["message"].encode()
    for alg, (name, _) in ALGS.items():
        if checked(alg, msg) != REFERENCE_KAT[name]:
            raise SystemExit(f"oracle fails the reference KAT for {name}")
    kat = {"reference": REFERENCE_KAT, "fips": {}, "boundary": {}, "hmac": []}
    for key, m in FIPS_MESSAGES.items():
        kat["fips"][key] = {name: checked(alg, m) for alg, (name, _) in ALGS.items()}
    for n in BOUNDARY_LENGTHS:
        m = pattern(n)
        kat["boundary"][str(n)] = {name: checked(alg, m)
                                   for alg, (name, _) in ALGS.items()}
    # HMAC rows (4..6): keys of exactly hashlen bytes, as the registry requires
    for alg, hname, hl in ((4, "sha256", 32), (5, "sha384", 48), (6, "sha512", 64)):
        for n in (0, 1, 55, 64, 111, 128, 1024, 1500):
            key = bytes(((5 * i + 11 * alg) & 0xFF) for i in range(hl))
            msg = pattern(n)
            d = oracle.hmac(alg, key, msg)
            if d != pyhmac.new(key, msg, hname).digest():
                raise SystemExit(f"oracle/hmac disagree: alg {alg} len {n}")
            kat["hmac"].append({"alg": alg, "key": key.hex(), "len": n,
                                "digest": d.hex()})
    return kat


def make_batches():
    """Seeded batches: inputs are regenerated from (seed, shape) by
    tests/synth.py; we store every digest's SHA-256 (checksum of checksums)
    plus the first and last digests."""
    out = []
    shapes = [
        ("fixed", 1, 2, 1024, 1024, 1024),   # C2 shape (small n)
        ("fixed", 3, 5, 1024, 1024, 1024),   # C4 shape, SHA-512
        ("fixed", 2, 5, 257, 1024, 1024),    # SHA-384
        ("fixed", 1, 7, 333, 1000, 1008),    # non-block-multiple, padded stride
        ("fixed", 1, 8, 64, 0, 16),          # empty packets
    ]
    for kind, alg, seed, n, length, stride in shapes:
        data = synth.fixed_batch(seed, n, length, stride)
        d = oracle.batch(alg, data, stride=stride, length=length, n=n)
        for i in (0, n - 1):
            msg = data[i * stride:i * stride + length].tobytes()
            assert d[i].tobytes() == ALGS[alg][1](msg).digest()
        out.append({"kind": kind, "alg": alg, "seed": seed, "n": n,
                    "len": length, "stride": stride,
                    "digest_of_digests": hashlib.sha256(d.tobytes()).hexdigest(),
                    "first": d[0].tobytes().hex(), "last": d[-1].tobytes().hex()})
    for alg, lseed, bseed, n, align in ((1, 3, 4, 4096, 1), (3, 3, 4, 2048, 1),
                                        (1, 9, 10, 1500, 16)):
        lens = synth.mixed_lengths(lseed, n)
        data, offs = synth.packed(bseed, lens, align=align)
        d = oracle.batch(alg, data, offsets=offs, lens=lens)
        for i in (0, n - 1):
            msg = data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
            assert d[i].tobytes() == ALGS[alg][1](msg).digest()
        out.append({"kind": "mixed", "alg": alg, "len_seed": lseed,
                    "seed": bseed, "n": n, "align": align,
                    "digest_of_digests": hashlib.sha256(d.tobytes()).hexdigest(),
                    "first": d[0].tobytes().hex(), "last": d[-1].tobytes().hex()})
    return out


def main():
    kat = make_kat()
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "batches.json"), "w") as f:
        json.dump(make_batches(), f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "kat.json"), os.path.join(HERE, "batches.json"))


if __name__ == "__main__":
    main()
