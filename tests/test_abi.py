"""CPU: the C-ABI library loads, exports every declared entry point, and the
host-only parts (registry, argument checks) behave like the reference's
call sites expect.  No kernel is launched here."""
import ctypes
import errno
import os
import re

import pytest

from ilias_net2_amd import _lib
from ilias_net2_amd import hash as h

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for hdr in ("sha2_batch.h", "hash.h", "packet.h", "sha2.h"):
        src = open(os.path.join(ROOT, "include", "net2", hdr)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"^#.*$", "", src, flags=re.M)
        names.update(re.findall(r"\b((?:net2_|SHA(?:256|384|512))\w+)\s*\(", src))
        names.update(re.findall(r"extern\s+const\s+int\s+(net2_\w+)\s*;", src))
    return names


def test_library_builds_and_loads():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    L = _lib.lib()
    assert L.net2_sha2_abi_version() == 1


def test_every_declared_symbol_exported():
    L = _lib.lib()
    decl = declared_symbols()
    assert {"net2_sha2_dev_fixed", "net2_sha2_dev_var", "net2_sha2_batch",
            "net2_hashctx_hashiov", "net2_hashmax", "SHA256Init",
            "SHA512Transform", "net2_sha2_ctx_update"} <= decl
    for name in decl:
        assert hasattr(L, name), name
    # and the binding declares them all
    assert decl == set(_lib.SIGNATURES) | set(_lib.DATA_SYMBOLS)


def test_registry_rows():
    # row 0 is nil (connection.c:336, packet.n2t:217 test alg != 0)
    assert h.hashmax() == 7
    assert [h.getname(i) for i in range(7)] == [
        "nil", "SHA256", "SHA384", "SHA512",
        "HMAC-SHA256", "HMAC-SHA384", "HMAC-SHA512"]
    assert h.getname(7) is None and h.getname(-1) is None
    for i in range(7):
        assert h.findname(h.getname(i)) == i
    assert h.findname("MD5") == -1
    assert [h.gethashlen(i) for i in range(7)] == [0, 32, 48, 64, 32, 48, 64]
    assert [h.getkeylen(i) for i in range(7)] == [0, 0, 0, 0, 32, 48, 64]
    assert h.gethashlen(99) == -1 and h.getkeylen(99) == -1


def _select_sighash(algs):
    """conn_negotiator.c:189-206 restated: longest unkeyed digest >= 4 B."""
    sel, best = -1, -1
    for a in algs:
        if h.getkeylen(a) != 0:
            continue
        hl = h.gethashlen(a)
        if hl >= 4 and hl > best:
            sel, best = a, hl
    return sel


def _select_hash(algs):
    """conn_negotiator.c:110-131 restated: keyed, key >= 16, hash >= 4."""
    sel, key, hsh = -1, -1, -1
    for a in algs:
        k, hl = h.getkeylen(a), h.gethashlen(a)
        if k >= 16 and hl >= 4 and (k > key or (k == key and hl > hsh)):
            sel, key, hsh = a, k, hl
    return sel


def test_negotiation_picks():
    assert _select_sighash(range(h.hashmax())) == 3      # SHA512
    assert _select_sighash([0, 1]) == 1                  # SHA256
    assert _select_sighash([0, 4, 5]) == -1              # keyed only
    assert _select_hash(range(h.hashmax())) == 6         # HMAC-SHA512
    assert _select_hash([1, 2, 3]) == -1


def test_argument_errors_without_launch():
    L = _lib.lib()
    buf = ctypes.create_string_buffer(64)
    # bad alg rows
    for alg in (-1, 0, 4, 7):
        assert L.net2_sha2_dev_fixed(alg, buf, 16, 16, 1, buf, None) == errno.EINVAL
        assert L.net2_sha2_batch(alg, buf, None, None, 16, 16, 1, buf, 0) == errno.EINVAL
    # n == 0 is a no-op even without a device
    assert L.net2_sha2_dev_fixed(1, None, 0, 0, 0, None, None) == 0
    # len > stride with several packets
    assert L.net2_sha2_dev_fixed(1, buf, 8, 16, 2, buf, None) == errno.EINVAL
    # var: workspace too small
    assert L.net2_sha2_dev_var(1, buf, buf, buf, 10, buf, buf, 4, None) == errno.EINVAL
    # hashiov: unkeyed row given a key (hash-openssl.cc:199-200), keyed row
    # with a wrong key size (hash-openssl.cc:101), short output
    iov = (_lib.IOVec * 1)(_lib.IOVec(ctypes.cast(buf, ctypes.c_void_p), 3))
    assert L.net2_hashctx_hashiov(1, buf, 4, iov, 1, buf, 64) == errno.EINVAL
    assert L.net2_hashctx_hashiov(4, buf, 16, iov, 1, buf, 64) == errno.EINVAL
    assert L.net2_hashctx_hashiov(3, None, 0, iov, 1, buf, 32) == errno.EINVAL
    assert L.net2_hashctx_hashiov(99, None, 0, iov, 1, buf, 64) == errno.EINVAL
    # nil hashes to nothing
    assert L.net2_hashctx_hashiov(0, None, 0, iov, 1, None, 0) == 0
    # streaming context: bad rows, NULL context (Init(NULL) is a no-op,
    # src/sha2.c:283), zero-length update is a no-op (:455)
    ctx = ctypes.create_string_buffer(208)
    assert L.net2_sha2_ctx_init(0, ctx) == errno.EINVAL
    assert L.net2_sha2_ctx_init(4, ctx) == errno.EINVAL
    assert L.net2_sha2_ctx_init(1, None) == 0
    L.SHA256Init(None)
    assert L.net2_sha2_ctx_update(1, None, buf, 1) == errno.EINVAL
    assert L.net2_sha2_ctx_init(3, ctx) == 0
    before = ctx.raw
    assert L.net2_sha2_ctx_update(3, ctx, None, 0) == 0
    assert ctx.raw == before
    assert L.net2_sha2_ctx_transform(2, None, buf) == errno.EINVAL


def test_factory_key_rules():
    with pytest.raises(ValueError):
        h.sha256().instantiate(b"k")
    with pytest.raises(ValueError):
        h.hmac_sha256().instantiate(b"short")
    f = h.sha512()
    assert (f.name, f.hashlen, f.keylen) == ("SHA512", 64, 0)


@pytest.mark.skipif(_lib.device_count() > 0, reason="a GPU is present")
def test_no_device_fails_loudly():
    """No CPU fallback: compute entry points report ENODEV."""
    L = _lib.lib()
    buf = ctypes.create_string_buffer(64)
    n = ctypes.c_int(-1)
    assert L.net2_sha2_device_count(ctypes.byref(n)) == errno.ENODEV
    assert n.value == 0
    assert L.net2_sha2_dev_fixed(1, buf, 16, 16, 1, buf, None) == errno.ENODEV
    assert L.net2_sha2_batch(1, buf, None, None, 16, 16, 1, buf, 0) == errno.ENODEV
    with pytest.raises(_lib.Net2Error) as ei:
        h.sha256().run(b"", b"abc")
    assert ei.value.errno == errno.ENODEV
    # the streaming context: buffering is host bookkeeping, a compression
    # needs the device (and the context is left as it was)
    ctx = ctypes.create_string_buffer(208)
    assert L.net2_sha2_ctx_init(1, ctx) == 0
    assert L.net2_sha2_ctx_update(1, ctx, buf, 10) == 0
    before = ctx.raw
    assert L.net2_sha2_ctx_update(1, ctx, buf, 64) == errno.ENODEV
    assert ctx.raw == before
    assert L.net2_sha2_ctx_final(1, buf, ctx) == errno.ENODEV
    # host-memory packet bursts: arguments checked first, then no device
    off = (ctypes.c_uint64 * 1)(0)
    ln = (ctypes.c_uint32 * 1)(16)
    key = b"k" * 64
    keys = _lib.BurstRxKeys(6, ctypes.cast(ctypes.c_char_p(key), ctypes.c_void_p),
                            64, 1, None, 0, 0, 0, 0)
    assert L.net2_packet_decode_burst_host(ctypes.byref(keys), 16, buf, off, ln, 1,
                                           buf, buf, None, None, 0) == errno.ENODEV
    assert L.net2_packet_decode_burst_host(ctypes.byref(keys), 65, buf, off, ln, 1,
                                           buf, buf, None, None, 0) == errno.EINVAL
    seq = (ctypes.c_uint32 * 1)(0)
    assert L.net2_packet_encode_burst_host(6, key, 64, 1, seq, seq, buf, off, ln, 1,
                                           buf, 0) == errno.ENODEV
    assert L.net2_packet_encode_burst_host(6, key, 63, 1, seq, seq, buf, off, ln, 1,
                                           buf, 0) == errno.EINVAL
    # the binning limits are host state; a workspace's counters need a device
    assert L.net2_sha2_bin_limits(0, -1) == 0
    st = _lib.BinStats()
    assert L.net2_sha2_workspace_stats(buf, 64, ctypes.byref(st)) == errno.EINVAL
    big = ctypes.create_string_buffer(L.net2_sha2_dev_var_workspace(0) + 8)
    aligned = (ctypes.addressof(big) + 7) & ~7
    assert L.net2_sha2_workspace_stats(aligned, L.net2_sha2_dev_var_workspace(0),
                                       ctypes.byref(st)) == errno.ENODEV
    # the thread's device selection: clearing it is host state and reports
    # the previous one; selecting a device needs one
    prev = ctypes.c_int(7)
    assert L.net2_sha2_set_device(-1, ctypes.byref(prev)) == 0 and prev.value == -1
    assert L.net2_sha2_set_device(0, None) == errno.ENODEV
    assert L.net2_sha2_get_device(None) == errno.EINVAL
    assert L.net2_sha2_get_device(ctypes.byref(prev)) == errno.ENODEV


def test_partial_abi_build_is_refused(tmp_path):
    """A build lacking entry points of this ABI (NET2_SHA2_LIB pointed at an
    older round's library) is refused, naming what it lacks, unless the A/B
    opt-in is set."""
    so = tmp_path / "libpartial.so"
    src = tmp_path / "partial.c"
    src.write_text("int net2_sha2_abi_version(void) { return 1; }\n")
    import subprocess
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    with pytest.raises(ImportError) as ei:
        _lib.bind(ctypes.CDLL(str(so)))
    assert "net2_sha2_batch" in str(ei.value)
    h2 = _lib.bind(ctypes.CDLL(str(so)), allow_old_abi=True)
    assert h2.net2_sha2_abi_version() == 1


@pytest.mark.skipif(_lib.device_count() > 0, reason="a GPU is present")
@pytest.mark.parametrize("call", ["SHA256Update", "SHA512Final", "SHA256Transform"])
def test_void_forms_abort_as_last_resort(call):
    """The reference's void SHA* calls cannot return an error, so a device
    failure inside one is fatal: it prints why and aborts rather than leave a
    wrong digest (the documented last resort).  Reference
    callers are bound to the errno-returning entry points instead, which
    report the same failure (test_no_device_fails_loudly).  Buffering a
    partial block needs no device and does not abort.  Fresh process each."""
    import subprocess
    import sys
    code = (
        "import ctypes, sys\n"
        "L = ctypes.CDLL(sys.argv[1])\n"
        "ctx = ctypes.create_string_buffer(208)\n"
        "L.SHA256Init(ctx); L.SHA512Init(ctx)\n"
        "L.SHA256Update(ctx, b'x' * 10, ctypes.c_size_t(10))\n"
        "print('PARTIAL-OK', flush=True)\n"
        "if sys.argv[2] == 'SHA256Update':\n"
        "    L.SHA256Init(ctx); L.SHA256Update(ctx, b'x' * 64, ctypes.c_size_t(64))\n"
        "elif sys.argv[2] == 'SHA512Final':\n"
        "    L.SHA512Init(ctx); L.SHA512Final(ctypes.create_string_buffer(64), ctx)\n"
        "else:\n"
        "    L.SHA256Transform(ctypes.create_string_buffer(32), b'y' * 64)\n"
        "print('RETURNED', flush=True)\n")
    r = subprocess.run([sys.executable, "-c", code, _lib.LIB_PATH, call],
                       capture_output=True, text=True, timeout=300)
    assert "PARTIAL-OK" in r.stdout, r.stdout + r.stderr
    assert "RETURNED" not in r.stdout
    assert r.returncode == -6, (r.returncode, r.stderr)   # SIGABRT
    assert f"net2: {call} failed on the GPU" in r.stderr, r.stderr
    assert "cannot report it" in r.stderr


def test_missing_library_fails_loudly():
    """No library, no hashing: the binding raises instead of falling back
    to any CPU path (checked in a fresh interpreter)."""
    import subprocess
    import sys
    env = dict(os.environ, NET2_SHA2_LIB="/nonexistent/libnet2_sha2.so")
    code = ("from ilias_net2_amd import hash as h\n"
            "try:\n"
            "    h.sha256().run(b'', b'x')\n"
            "except ImportError as e:\n"
            "    print('IMPORTERROR', e)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert "IMPORTERROR" in r.stdout and "no CPU fallback" in r.stdout, r.stdout + r.stderr


def test_build_id_is_the_device_code_hash(tmp_path):
    """net2_sha2_build_id() -- the stamp profiles/pmc_*.json carry and
    bench.py checks -- is the SHA-256 (16 hex digits) of the device code
    actually linked into the library (its .hip_fatbin section)."""
    import hashlib
    import shutil
    import subprocess
    objcopy = "/opt/rocm/lib/llvm/bin/llvm-objcopy"
    if not os.path.exists(objcopy):
        pytest.skip("no llvm-objcopy")
    fat = tmp_path / "lib.fatbin"
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fat}", _lib.LIB_PATH,
                    str(tmp_path / "copy.so")], check=True, capture_output=True)
    want = hashlib.sha256(fat.read_bytes()).hexdigest()[:16]
    assert _lib.lib().net2_sha2_build_id().decode() == want
    shutil.rmtree(tmp_path, ignore_errors=True)
