"""ctypes binding of libnet2_sha2.so, the C-ABI of the MI355X SHA-2 path.

The binding declares exactly the entry points of include/net2/sha2_batch.h,
include/net2/hash.h, include/net2/packet.h and include/net2/sha2.h.  Loading is strict: if the shared library is missing the
import of any compute helper raises, there is no Python or CPU fallback.
"""
from __future__ import annotations

import ctypes
import errno
import os

LIB_NAME = "libnet2_sha2.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# Build-variant A/B runs (tools/gpu_ab_lib.sh) point this at another build of
# the same library; unset, the in-tree library is the one loaded.  A build
# lacking an entry point of this ABI is refused unless
# NET2_SHA2_LIB_ALLOW_OLD_ABI=1 (bind()).
LIB_PATH = os.environ.get("NET2_SHA2_LIB", LIB_PATH)

# Registry rows (include/net2/sha2_batch.h, include/net2/hash.h).
NIL, SHA256, SHA384, SHA512 = 0, 1, 2, 3
HMAC_SHA256, HMAC_SHA384, HMAC_SHA512 = 4, 5, 6
DIGEST_LEN = {SHA256: 32, SHA384: 48, SHA512: 64,
              HMAC_SHA256: 32, HMAC_SHA384: 48, HMAC_SHA512: 64}
BLOCK_LEN = {SHA256: 64, SHA384: 128, SHA512: 128}


class Net2Error(OSError):
    """A non-zero errno-style return from the C ABI."""


class IOVec(ctypes.Structure):
    _fields_ = [("iov_base", ctypes.c_void_p), ("iov_len", ctypes.c_size_t)]


class BurstRxKeys(ctypes.Structure):
    """struct net2_burst_rx_keys (include/net2/packet.h)."""
    _fields_ = [("hash_alg", ctypes.c_int), ("hash_key", ctypes.c_void_p),
                ("hash_keylen", ctypes.c_size_t), ("enc_alg", ctypes.c_int),
                ("alt_hash_key", ctypes.c_void_p),
                ("alt_hash_keylen", ctypes.c_size_t),
                ("alt_no_cutoff", ctypes.c_int), ("alt_cutoff", ctypes.c_uint32),
                ("rx_start", ctypes.c_uint32)]


class BinStats(ctypes.Structure):
    """struct net2_bin_stats (include/net2/sha2_batch.h)."""
    _fields_ = [("prepared", ctypes.c_uint32), ("binned", ctypes.c_uint32),
                ("aborts", ctypes.c_uint32), ("mismatches", ctypes.c_uint32),
                ("unprepared", ctypes.c_uint32)]


_c_u64p = ctypes.POINTER(ctypes.c_uint64)
_c_u32p = ctypes.POINTER(ctypes.c_uint32)

# name -> (restype, argtypes)
SIGNATURES = {
    "net2_sha2_abi_version": (ctypes.c_int, []),
    "net2_sha2_build_id": (ctypes.c_char_p, []),
    "net2_sha2_numa_stats": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p]),
    "net2_sha2_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "net2_sha2_set_device": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "net2_sha2_get_device": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "net2_sha2_last_hip_error": (ctypes.c_int, []),
    "net2_sha2_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "net2_sha2_dev_fixed": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "net2_sha2_dev_var": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
        ctypes.c_void_p]),
    "net2_sha2_dev_var_workspace": (ctypes.c_size_t, [ctypes.c_uint64]),
    "net2_sha2_workspace_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t,
                                                ctypes.c_void_p]),
    "net2_sha2_workspace_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t,
                                                 ctypes.c_void_p]),
    "net2_sha2_bin_limits": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_int64]),
    "net2_sha2_burst_limits": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64]),
    "net2_sha2_batch": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
        ctypes.c_int]),
    "net2_hash_getname": (ctypes.c_char_p, [ctypes.c_int]),
    "net2_hash_findname": (ctypes.c_int, [ctypes.c_char_p]),
    "net2_hash_gethashlen": (ctypes.c_int, [ctypes.c_int]),
    "net2_hash_getkeylen": (ctypes.c_int, [ctypes.c_int]),
    "net2_hashctx_hashiov": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
        ctypes.POINTER(IOVec), ctypes.c_size_t, ctypes.c_void_p,
        ctypes.c_size_t]),
    "net2_coalesce_stats": (ctypes.c_int, [
        ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
        ctypes.POINTER(ctypes.c_uint64)]),
    "net2_hmac_dev": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
        ctypes.c_void_p]),
    "net2_hmac_sign_dev": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
        ctypes.c_size_t, ctypes.c_void_p]),
    "net2_hmac_verify_dev": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "net2_ph_to_iv_buf": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_void_p]),
    "net2_ph_to_iv_dev": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_void_p, ctypes.c_void_p]),
    "net2_packet_burst_workspace": (ctypes.c_size_t, [ctypes.c_uint64]),
    "net2_packet_decode_burst": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
        ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "net2_packet_decode_burst_ck": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
        ctypes.c_void_p]),
    "net2_packet_encode_burst": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_size_t, ctypes.c_void_p]),
    "net2_packet_decode_burst_host": (ctypes.c_int, [
        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "net2_packet_encode_burst_host": (ctypes.c_int, [
        ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]),
    # include/net2/sha2.h: the streaming interface of src/sha2.c
    "net2_sha2_ctx_init": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p]),
    "net2_sha2_ctx_update": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_size_t]),
    "net2_sha2_ctx_pad": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p]),
    "net2_sha2_ctx_final": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "net2_sha2_ctx_transform": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p,
                                               ctypes.c_void_p]),
}
for _pfx in ("SHA256", "SHA384", "SHA512"):
    SIGNATURES[_pfx + "Init"] = (None, [ctypes.c_void_p])
    SIGNATURES[_pfx + "Update"] = (None, [ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t])
    SIGNATURES[_pfx + "Pad"] = (None, [ctypes.c_void_p])
    SIGNATURES[_pfx + "Final"] = (None, [ctypes.c_void_p, ctypes.c_void_p])
    SIGNATURES[_pfx + "Transform"] = (None, [ctypes.c_void_p, ctypes.c_void_p])
DATA_SYMBOLS = ("net2_hashmax",)

_lib = None


def _share_torch_hip_runtime() -> None:
    """One HIP runtime per process.

    PyTorch wheels bundle their own libamdhip64.so (SONAME libamdhip64.so.7,
    the same SONAME as /opt/rocm's).  If torch is loaded first, the dynamic
    linker satisfies this library's DT_NEEDED with torch's copy and the
    process has one runtime; if this library came first, torch would load a
    second runtime and lose the device.  So when torch is importable, import
    it before dlopen-ing libnet2_sha2.so.  Pure C callers are unaffected."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> ctypes.CDLL:
    """The loaded C ABI; raises if the HIP library was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` "
                "(there is no CPU fallback for the SHA-2 path)")
        _share_torch_hip_runtime()
        _lib = bind(ctypes.CDLL(LIB_PATH),
                    allow_old_abi=os.environ.get("NET2_SHA2_LIB_ALLOW_OLD_ABI") == "1")
    return _lib


def bind(handle: ctypes.CDLL, allow_old_abi: bool = False) -> ctypes.CDLL:
    """Declare every SIGNATURES entry on a loaded build of the library.

    A missing symbol raises, naming every one missing, unless allow_old_abi
    (NET2_SHA2_LIB_ALLOW_OLD_ABI=1: an A/B build of an earlier round, whose
    ABI may lack later entry points; the names skipped are logged)."""
    missing = [name for name in SIGNATURES if not hasattr(handle, name)]
    if missing and not allow_old_abi:
        raise ImportError(f"{handle._name} lacks {len(missing)} entry point(s) of "
                          f"this ABI: {', '.join(missing)} (an older build? set "
                          "NET2_SHA2_LIB_ALLOW_OLD_ABI=1 for A/B runs)")
    if missing:
        import sys
        print(f"_lib: {handle._name}: older ABI, not bound: {', '.join(missing)}",
              file=sys.stderr, flush=True)
    for name, (res, args) in SIGNATURES.items():
        if name in missing:
            continue
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    return handle


def strerror(rc: int) -> str:
    return lib().net2_sha2_strerror(rc).decode()


def check(rc: int, what: str = "") -> None:
    """Raise Net2Error for a non-zero return code."""
    if rc != 0:
        msg = strerror(rc)
        if rc == errno.EIO:
            msg += f" (hip error {lib().net2_sha2_last_hip_error()})"
        raise Net2Error(rc, f"{what}: {msg}" if what else msg)


def hashmax() -> int:
    return ctypes.c_int.in_dll(lib(), "net2_hashmax").value


def workspace_stats(ws_ptr: int, ws_bytes: int) -> dict:
    """net2_sha2_workspace_stats of a device workspace, as a dict."""
    st = BinStats()
    check(lib().net2_sha2_workspace_stats(ws_ptr, ws_bytes, ctypes.byref(st)),
          "net2_sha2_workspace_stats")
    return {f: getattr(st, f) for f, _ in BinStats._fields_}


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().net2_sha2_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0
