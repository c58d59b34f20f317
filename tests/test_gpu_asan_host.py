"""GPU: the library's host code under AddressSanitizer (tests/asan/).

`make -C tests/asan` rebuilds every object of libnet2_sha2 with ASan on the
host side only (`-Xarch_host -fsanitize=address`; the gfx950 code objects
are the shipped ones) and links them with the CPU oracle into
`tests/asan/host_asan`, which drives net2_sha2_batch, both host bursts and
concurrent single calls through the C ABI and checks every output against
the oracle (see its header).  A heap / stack / global overflow, a use after
free in our host code aborts it (leak checking at exit is off on the GPU:
see _env).  Run once on the real
device count and once with three virtual devices, so the sharded paths
(one slice per device, persistent slice workers) run under ASan too.
`tests/asan/test_sign_asan` does the same for the host C layer of the
signed-payload callers (csrc/host/*.c) through tests/c/test_sign.c.
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "asan", "host_asan")
SIGN = os.path.join(HERE, "asan", "test_sign_asan")
KEYS = [os.path.join(HERE, "golden", "keys", f)
        for f in ("ecdsa_p521_priv.pem", "ecdsa_p521_pub.pem")]


def _env(virtual=None):
    env = dict(os.environ)
    # Leak checking at exit is off here: LeakSanitizer stops every thread of
    # the process at exit, and with the HIP runtime's threads in some states
    # that never returned (2 of 3 runs of tools/asan_hang_probe.sh hung after
    # "host_asan ok" was due, 0 of 3 with detect_leaks=0).  Address errors
    # still abort the run.
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:halt_on_error=1"
    env["LSAN_OPTIONS"] = "suppressions=" + os.path.join(HERE, "asan", "lsan.supp")
    env.pop("NET2_SHA2_VIRTUAL_DEVICES", None)
    if virtual:
        env["NET2_SHA2_VIRTUAL_DEVICES"] = virtual
    return env


@pytest.mark.gpu
@pytest.mark.parametrize("virtual", [None, "3"])
def test_host_code_under_asan(virtual):
    if not os.path.exists(EXE):
        pytest.skip("tests/asan/host_asan not built (make -C tests/asan)")
    run = subprocess.run([EXE], capture_output=True, text=True, env=_env(virtual),
                         timeout=300)
    out = run.stdout + run.stderr
    print(out[-3000:])
    assert run.returncode == 0, out[-6000:]
    assert "host_asan ok" in run.stdout
    assert "AddressSanitizer" not in out


@pytest.mark.gpu
def test_signed_payload_layer_under_asan():
    """tests/c/test_sign.c (the reference's test/sign.c restated, parts 1-3:
    fingerprints, signature create / validate single and batched, the
    signed-carver tick at 4096 x 1 KiB with its helper pool) over the host C
    layer and the library, both built with ASan."""
    if not os.path.exists(SIGN):
        pytest.skip("tests/asan/test_sign_asan not built (make -C tests/asan)")
    run = subprocess.run([SIGN, *KEYS], capture_output=True, text=True, env=_env(),
                         timeout=300)
    out = run.stdout + run.stderr
    print(out[-3000:])
    assert run.returncode == 0, out[-6000:]
    assert "PASS (0 failures)" in run.stdout
    assert "AddressSanitizer" not in out
