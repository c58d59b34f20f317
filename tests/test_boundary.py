"""CPU: the product never hashes on the CPU and never touches the oracle.

The shipped libraries (libnet2_sha2.so, libnet2_sign.so, libnet2_hash_cxx.so)
must not link the oracle or any CPU SHA-2 / HMAC implementation (OpenSSL's
digest and MAC entry points): every digest they produce comes from the HIP
kernels.  The Python package must not import the oracle either.  (The oracle
is test infrastructure: tests/, smoke() and bench.py's cpu_baseline only.)
"""
import ast
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ilias_net2_amd")
LIBS = ["libnet2_sha2.so", "libnet2_sign.so", "libnet2_hash_cxx.so"]
# OpenSSL entry points that would hash on the CPU
CPU_HASH = re.compile(r"^(SHA(1|224|256|384|512)\w*|EVP_(Digest\w*|sha\w+|MD_\w+|MAC_\w+|Q_digest)|"
                      r"HMAC\w*|EVP_MD_CTX\w*)$")


def _tool(name):
    path = shutil.which(name)
    if path is None:
        pytest.skip(f"{name} not available")
    return path


@pytest.mark.parametrize("lib", LIBS)
def test_no_oracle_no_cpu_sha(lib):
    path = os.path.join(PKG, lib)
    if not os.path.exists(path):
        pytest.fail(f"{lib} not built (run __graft_entry__.build())")
    dyn = subprocess.run([_tool("readelf"), "-d", path], capture_output=True,
                         text=True, check=True).stdout
    needed = re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", dyn)
    assert needed, dyn
    assert not [n for n in needed if "oracle" in n], needed
    if lib == "libnet2_sha2.so":
        # the hashing library links the HIP runtime, not a crypto library
        assert not [n for n in needed if "crypto" in n or "ssl" in n], needed
        assert "libamdhip64.so.7" in needed or any("amdhip64" in n for n in needed), needed
    und = subprocess.run([_tool("nm"), "-D", "--undefined-only", path],
                         capture_output=True, text=True, check=True).stdout
    syms = [ln.split()[-1] for ln in und.splitlines() if ln.strip()]
    assert not [s for s in syms if s.startswith("oracle_")], syms
    cpu = [s for s in syms if CPU_HASH.match(s.split("@")[0])]
    assert not cpu, f"{lib} references CPU hash functions: {cpu}"


def test_package_does_not_import_oracle():
    for dirpath, _, files in os.walk(PKG):
        for f in files:
            if not f.endswith(".py"):
                continue
            path = os.path.join(dirpath, f)
            with open(path) as fh:
                tree = ast.parse(fh.read(), path)
            for node in ast.walk(tree):
                names = []
                if isinstance(node, ast.Import):
                    names = [a.name for a in node.names]
                elif isinstance(node, ast.ImportFrom):
                    names = [node.module or ""]
                assert not [n for n in names if n.split(".")[0] == "oracle"], (path, names)
