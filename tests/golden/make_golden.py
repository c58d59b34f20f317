"""Regenerate the golden vectors under tests/golden/.

Sources, in order of authority:
  1. the reference's own known-answer tests, test/hash.cc:21-48 (SHA-256/384/
     512 of "Luke, I am your father."), copied here as data;
  2. FIPS 180-4 / NIST CAVP example messages ("abc", "", the 448- and 896-bit
     messages, one million 'a'), and the RFC 4231 HMAC-SHA-256/384/512 test
     cases 1-7 (published MACs, every key length incl. > block size);
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

# RFC 4231 section 4 (HMAC-SHA-256/384/512 test cases 1-7), the published
# values as data.  Case 5's MACs are truncated to 128 bits by the RFC.
RFC4231 = [
    {"case": 1, "key": "0b" * 20, "data": b"Hi There".hex(),
     "HMAC-SHA256": "b0344c61d8db38535ca8afceaf0bf12b881dc200c9833da726e9376c2e32cff7",
     "HMAC-SHA384": ("afd03944d84895626b0825f4ab46907f15f9dadbe4101ec682aa034c7cebc59c"
                     "faea9ea9076ede7f4af152e8b2fa9cb6"),
     "HMAC-SHA512": ("87aa7cdea5ef619d4ff0b4241a1d6cb02379f4e2ce4ec2787ad0b30545e17cde"
                     "daa833b7d6b8a702038b274eaea3f4e4be9d914eeb61f1702e696c203a126854")},
    {"case": 2, "key": b"Jefe".hex(), "data": b"what do ya want for nothing?".hex(),
     "HMAC-SHA256": "5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843",
     "HMAC-SHA384": ("af45d2e376484031617f78d2b58a6b1b9c7ef464f5a01b47e42ec3736322445e"
                     "8e2240ca5e69e2c78b3239ecfab21649"),
     "HMAC-SHA512": ("164b7a7bfcf819e2e395fbe73b56e0a387bd64222e831fd610270cd7ea250554"
                     "9758bf75c05a994a6d034f65f8f0e6fdcaeab1a34d4a6b4b636e070a38bce737")},
    {"case": 3, "key": "aa" * 20, "data": "dd" * 50,
     "HMAC-SHA256": "773ea91e36800e46854db8ebd09181a72959098b3ef8c122d9635514ced565fe",
     "HMAC-SHA384": ("88062608d3e6ad8a0aa2ace014c8a86f0aa635d947ac9febe83ef4e55966144b"
                     "2a5ab39dc13814b94e3ab6e101a34f27"),
     "HMAC-SHA512": ("fa73b0089d56a284efb0f0756c890be9b1b5dbdd8ee81a3655f83e33b2279d39"
                     "bf3e848279a722c806b485a47e67c807b946a337bee8942674278859e13292fb")},
    {"case": 4, "key": bytes(range(1, 26)).hex(), "data": "cd" * 50,
     "HMAC-SHA256": "82558a389a443c0ea4cc819899f2083a85f0faa3e578f8077a2e3ff46729665b",
     "HMAC-SHA384": ("3e8a69b7783c25851933ab6290af6ca77a9981480850009cc5577c6e1f573b4e"
                     "6801dd23c4a7d679ccf8a386c674cffb"),
     "HMAC-SHA512": ("b0ba465637458c6990e5a8c5f61d4af7e576d97ff94b872de76f8050361ee3db"
                     "a91ca5c11aa25eb4d679275cc5788063a5f19741120c4f2de2adebeb10a298dd")},
    {"case": 5, "key": "0c" * 20, "data": b"Test With Truncation".hex(),
     "HMAC-SHA256": "a3b6167473100ee06e0c796c2955552b",
     "HMAC-SHA384": "3abf34c3503b2a23a46efc619baef897",
     "HMAC-SHA512": "415fad6271580a531d4179bc891d87a6"},
    {"case": 6, "key": "aa" * 131,
     "data": b"Test Using Larger Than Block-Size Key - Hash Key First".hex(),
     "HMAC-SHA256": "60e431591ee0b67f0d8a26aacbf5b77f8e0bc6213728c5140546040f0ee37f54",
     "HMAC-SHA384": ("4ece084485813e9088d2c63a041bc5b44f9ef1012a2b588f3cd11f05033ac4c6"
                     "0c2ef6ab4030fe8296248df163f44952"),
     "HMAC-SHA512": ("80b24263c7c1a3ebb71493c1dd7be8b49b46d1f41b4aeec1121b013783f8f352"
                     "6b56d037e05f2598bd0fd2215d6a1e5295e64f73f63f0aec8b915a985d786598")},
    {"case": 7, "key": "aa" * 131,
     "data": (b"This is a test using a larger than block-size key and a larger "
              b"than block-size data. The key needs to be hashed before being "
              b"used by the HMAC algorithm.").hex(),
     "HMAC-SHA256": "9b09ffa71b942fcb27635fbcd5b0e944bfdc63644f0713938a7f51535c3a35e2",
     "HMAC-SHA384": ("6617178e941f020d351e2f254e8fd32c602420feb0b8fb9adccebb82461e99c5"
                     "a678cc31e799176d3860e6110c46523e"),
     "HMAC-SHA512": ("e37b6a775dc87dbaa4dfa9f96e5e3ffddebd71f8867289865df5a32d20cdc944"
                     "b6022cac3c4982b10d5eeb55c3e4de15134676fb6de0446065c97440fa8c6a58")},
]

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
    # RFC 4231: the oracle must reproduce every published MAC (and so must
    # Python's hmac, an independent implementation)
    for v in RFC4231:
        key, data = bytes.fromhex(v["key"]), bytes.fromhex(v["data"])
        for alg, hname in ((4, "sha256"), (5, "sha384"), (6, "sha512")):
            want = v["HMAC-" + hname.upper()]
            d = oracle.hmac(alg, key, data).hex()[:len(want)]
            p = pyhmac.new(key, data, hname).hexdigest()[:len(want)]
            if d != want or p != want:
                raise SystemExit(f"RFC 4231 case {v['case']} {hname}: "
                                 f"oracle {d == want}, hmac {p == want}")
    kat["rfc4231"] = RFC4231
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
