"""The MI355X backend of the reference's C++ hash interface
(include/ilias/net2/hash.h:31-79; ilias_net2_amd/csrc/cxx/hash_mi355x.cc),
exercised by tests/cxx/test_hash.cc, which restates the reference's own
test/hash.cc:50-80 (KATs through run() and instantiate/update/final) plus the
key rules of cxx_src/hash-openssl.cc and oracle cross-checks."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cxx", "test_hash")
LIB = os.path.join(ROOT, "ilias_net2_amd", "libnet2_hash_cxx.so")

FACTORIES = ("sha256", "sha384", "sha512", "hmac_sha256", "hmac_sha384",
             "hmac_sha512")


def test_backend_exports_the_factories():
    """The six factories of namespace ilias::hash (hash.h:73-79), by their
    C++ symbol names, so the reference's callers link against them."""
    r = subprocess.run(["nm", "-D", "-C", "--defined-only", LIB],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    for f in FACTORIES:
        assert f"ilias::hash::{f}()" in r.stdout, f


@pytest.mark.skipif(__import__("ilias_net2_amd._lib", fromlist=["x"]).device_count() > 0,
                    reason="a GPU is present")
def test_no_device_throws():
    """Without a device the backend throws (no CPU fallback)."""
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "no usable gfx950" in r.stderr


@pytest.mark.gpu
def test_reference_hash_cc_on_gpu():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "test_hash: ok" in r.stdout
    # the reference test's own output lines (test/hash.cc:55-62)
    for name in ("SHA256", "SHA384", "SHA512"):
        assert f"Test algorithm: {name}" in r.stdout
