"""CPU: wire encodings of net2x_signature (types/signature.n2t:48-53) and
signed_carver_header (types/signed_carver_header.n2t:21-43).

The byte layout is restated independently here from the reference's
surviving encoder, cxx_src/cp.cc:20-104 (u32 big-endian length, payload,
zero padding to a multiple of 8 including the length) and cp.h:178-205
(big-endian integers); the C encoder must produce exactly these bytes."""
import ctypes
import errno
import os
import struct

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Sig(ctypes.Structure):
    _fields_ = [("sign_alg", ctypes.c_char_p), ("hash_alg", ctypes.c_char_p),
                ("data", ctypes.POINTER(ctypes.c_uint8)), ("datalen", ctypes.c_size_t)]


class Hdr(ctypes.Structure):
    _fields_ = [("pl_segs", ctypes.c_uint16), ("sig_segs", ctypes.c_uint16)]


def _lib():
    import ilias_net2_amd._lib as L
    L.lib()
    lib = ctypes.CDLL(os.path.join(ROOT, "ilias_net2_amd", "libnet2_sign.so"))
    lib.net2x_signature_encoded_len.restype = ctypes.c_size_t
    lib.net2x_signature_deinit.restype = None
    return lib


def ref_field(b: bytes) -> bytes:
    """cxx_src/cp.cc: pad = 7 - (3 + len) % 8."""
    pad = 7 - (3 + len(b)) % 8
    return struct.pack(">I", len(b)) + b + b"\0" * pad


def ref_signature(sign_alg: bytes, hash_alg: bytes, data: bytes) -> bytes:
    return ref_field(sign_alg) + ref_field(hash_alg) + ref_field(data)


def test_signature_encode_matches_reference_layout():
    lib = _lib()
    rng = np.random.default_rng(1)
    for n in list(range(0, 20)) + [139, 1000]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for sa, ha in ((b"ecdsa", b"SHA512"), (b"", b"SHA256"), (b"abcdefg", b"")):
            buf = (ctypes.c_uint8 * max(n, 1)).from_buffer_copy(data or b"\0")
            s = Sig(sa, ha, buf, n)
            want = ref_signature(sa, ha, data)
            assert len(want) % 8 == 0
            assert lib.net2x_signature_encoded_len(ctypes.byref(s)) == len(want)
            out = ctypes.create_string_buffer(len(want))
            olen = ctypes.c_size_t(len(want))
            assert lib.net2x_signature_encode(ctypes.byref(s), out, ctypes.byref(olen)) == 0
            assert out.raw[:olen.value] == want
            # decode round trip
            d = Sig()
            used = ctypes.c_size_t(0)
            enc = want + b"trailing"
            assert lib.net2x_signature_decode(ctypes.byref(d), enc, len(enc), ctypes.byref(used)) == 0
            assert used.value == len(want)
            assert (d.sign_alg or b"") == sa and (d.hash_alg or b"") == ha
            assert bytes(d.data[:d.datalen]) == data
            lib.net2x_signature_deinit(ctypes.byref(d))


def test_signature_decode_rejects_malformed():
    lib = _lib()
    good = ref_signature(b"ecdsa", b"SHA512", b"\x01\x02\x03")
    d = Sig()
    used = ctypes.c_size_t()
    for bad in (good[:-1], good[:3], b"", good[:9] + b"\x01" + good[10:]):
        assert lib.net2x_signature_decode(ctypes.byref(d), bad, len(bad), ctypes.byref(used)) == errno.EINVAL
    huge = struct.pack(">I", 0xFFFFFFF0) + b"\0" * 12
    assert lib.net2x_signature_decode(ctypes.byref(d), huge, len(huge), ctypes.byref(used)) == errno.EINVAL
    small = ctypes.c_size_t(3)
    s = Sig(b"ecdsa", b"SHA512", None, 0)
    out = ctypes.create_string_buffer(64)
    assert lib.net2x_signature_encode(ctypes.byref(s), out, ctypes.byref(small)) == errno.EINVAL


def test_signed_carver_header():
    lib = _lib()
    for pl, sg in ((0, 0), (1, 2), (0xFFFF, 0x1234)):
        out = (ctypes.c_uint8 * 4)()
        lib.net2_signed_carver_header_encode(ctypes.byref(Hdr(pl, sg)), out)
        assert bytes(out) == struct.pack(">HH", pl, sg)
        h = Hdr()
        lib.net2_signed_carver_header_decode(ctypes.byref(h), out)
        assert (h.pl_segs, h.sig_segs) == (pl, sg)
