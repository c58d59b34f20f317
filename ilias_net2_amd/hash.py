"""Host mirror of the reference's hash interfaces over the MI355X C ABI.

Two reference surfaces are mirrored, with the same names, argument meaning
and error behaviour:

* the C registry (reconstructed, include/net2/hash.h): ``getname``,
  ``findname``, ``gethashlen``, ``getkeylen``, ``hashmax`` and ``hashbuf``
  (``net2_hashctx_hashbuf``, types/signature.n2t:92,147);
* the C++ factories of include/ilias/net2/hash.h:31-79 --
  ``sha256()``, ``sha384()``, ``sha512()``, ``hmac_sha256()`` ... returning a
  ``HashCtxFactory`` with ``name``, ``hashlen``, ``keylen``,
  ``instantiate(key)`` -> ``HashCtx`` (``update``/``final``) and
  ``run(key, data)``.  As in cxx_src/hash-openssl.cc:199-200,227-228 an
  unkeyed hash given a non-empty key raises ``ValueError`` (the
  ``std::invalid_argument`` of the C++ code), and a keyed hash needs a key of
  exactly ``keylen`` bytes (hash-openssl.cc:101).

Every digest is computed on the GPU: ``run``/``hashbuf`` through
``net2_hashctx_hashiov`` (one coalesced request), ``instantiate`` through the
streaming SHA2_CTX calls of net2/sha2.h; with no usable device the calls raise
``Net2Error(ENODEV)``.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Union

from . import _lib
from ._lib import IOVec, Net2Error  # noqa: F401  (re-exported)

Bytes = Union[bytes, bytearray, memoryview]


def hashmax() -> int:
    return _lib.hashmax()


def getname(alg: int):
    n = _lib.lib().net2_hash_getname(alg)
    return None if n is None else n.decode()


def findname(name: str) -> int:
    return _lib.lib().net2_hash_findname(name.encode())


def gethashlen(alg: int) -> int:
    return _lib.lib().net2_hash_gethashlen(alg)


def getkeylen(alg: int) -> int:
    return _lib.lib().net2_hash_getkeylen(alg)


def _iovecs(segments: Iterable[Bytes]):
    keep: List[object] = []
    vec: List[IOVec] = []
    for seg in segments:
        b = bytes(seg)
        buf = ctypes.create_string_buffer(b, len(b)) if b else None
        keep.append(buf)
        vec.append(IOVec(ctypes.cast(buf, ctypes.c_void_p) if buf else None,
                         len(b)))
    arr = (IOVec * max(len(vec), 1))(*vec)
    return arr, len(vec), keep


def hashbuf(alg: int, key: Bytes, data: Union[Bytes, Iterable[Bytes]]) -> bytes:
    """net2_hashctx_hashbuf: digest of data (bytes or a list of segments)."""
    segs = [data] if isinstance(data, (bytes, bytearray, memoryview)) else list(data)
    arr, cnt, keep = _iovecs(segs)
    hl = gethashlen(alg)
    if hl < 0:
        raise Net2Error(22, f"bad hash alg {alg}")
    out = ctypes.create_string_buffer(max(hl, 1))
    kb = bytes(key) if key else b""
    kbuf = ctypes.create_string_buffer(kb, len(kb)) if kb else None
    rc = _lib.lib().net2_hashctx_hashiov(alg, kbuf, len(kb), arr, cnt, out,
                                         len(out))
    del keep
    _lib.check(rc, f"net2_hashctx_hashiov({getname(alg)})")
    return out.raw[:hl]


class HashCtx:
    """ilias::hash_ctx (include/ilias/net2/hash.h:31-45), streaming: a
    SHA2_CTX of net2/sha2.h (src/sha2.c's context) whose compressions run on
    the GPU as update() completes blocks; keyed rows keep an inner context
    primed with K' ^ ipad and run the outer hash at final() (RFC 2104), as
    the C++ backend does (ilias_net2_amd/csrc/cxx/hash_mi355x.cc)."""

    _SHA_ROW = {1: 1, 2: 2, 3: 3, 4: 1, 5: 2, 6: 3}

    def __init__(self, factory: "HashCtxFactory", key: bytes):
        self.name = factory.name
        self.hashlen = factory.hashlen
        self.keylen = factory.keylen
        self._sha = self._SHA_ROW[factory.alg]
        self._blk = 64 if self._sha == 1 else 128
        self._ctx = ctypes.create_string_buffer(208)
        self._kpad = bytes(key) + b"\0" * (self._blk - len(key))
        self._done = False
        L = _lib.lib()
        _lib.check(L.net2_sha2_ctx_init(self._sha, self._ctx), "SHA2 init")
        if self.keylen:
            ipad = bytes(b ^ 0x36 for b in self._kpad)
            self._update(ipad)

    def _update(self, b: bytes) -> None:
        buf = ctypes.create_string_buffer(b, max(len(b), 1))
        _lib.check(_lib.lib().net2_sha2_ctx_update(self._sha, self._ctx, buf,
                                                   len(b)), "SHA2 update")

    def update(self, data: Bytes) -> None:
        if self._done:
            raise RuntimeError("hash_ctx already finalized")
        self._update(bytes(data))

    def final(self) -> bytes:
        if self._done:
            raise RuntimeError("hash_ctx already finalized")
        self._done = True
        L = _lib.lib()
        out = ctypes.create_string_buffer(64)
        _lib.check(L.net2_sha2_ctx_final(self._sha, out, self._ctx), "SHA2 final")
        if not self.keylen:
            return out.raw[:self.hashlen]
        inner = out.raw[:self.hashlen]
        _lib.check(L.net2_sha2_ctx_init(self._sha, self._ctx), "HMAC final")
        self._update(bytes(b ^ 0x5C for b in self._kpad))
        self._update(inner)
        _lib.check(L.net2_sha2_ctx_final(self._sha, out, self._ctx), "HMAC final")
        return out.raw[:self.hashlen]


class HashCtxFactory:
    """ilias::hash_ctx_factory (include/ilias/net2/hash.h:49-67)."""

    def __init__(self, alg: int):
        self.alg = alg
        self.name = getname(alg)
        self.hashlen = gethashlen(alg)
        self.keylen = getkeylen(alg)

    def _check_key(self, key: Bytes) -> bytes:
        key = bytes(key or b"")
        if self.keylen == 0 and key:
            raise ValueError("expected empty key buffer for un-keyed hash")
        if self.keylen and len(key) != self.keylen:
            raise ValueError(
                f"{self.name} needs a {self.keylen}-byte key, got {len(key)}")
        return key

    def instantiate(self, key: Bytes = b"") -> HashCtx:
        return HashCtx(self, self._check_key(key))

    def run(self, key: Bytes, data: Union[Bytes, Iterable[Bytes]]) -> bytes:
        return hashbuf(self.alg, self._check_key(key), data)

    def __repr__(self) -> str:
        return f"HashCtxFactory({self.name!r}, hashlen={self.hashlen}, keylen={self.keylen})"


def sha256() -> HashCtxFactory:
    return HashCtxFactory(_lib.SHA256)


def sha384() -> HashCtxFactory:
    return HashCtxFactory(_lib.SHA384)


def sha512() -> HashCtxFactory:
    return HashCtxFactory(_lib.SHA512)


def hmac_sha256() -> HashCtxFactory:
    return HashCtxFactory(_lib.HMAC_SHA256)


def hmac_sha384() -> HashCtxFactory:
    return HashCtxFactory(_lib.HMAC_SHA384)


def hmac_sha512() -> HashCtxFactory:
    return HashCtxFactory(_lib.HMAC_SHA512)
