"""GPU: the library's host code under AddressSanitizer (tests/asan/).

`make -C tests/asan` rebuilds every object of libnet2_sha2 with ASan on the
host side only (`-Xarch_host -fsanitize=address`; the gfx950 code objects
are the shipped ones) and links them with the CPU oracle into
`tests/asan/host_asan`, which drives net2_sha2_batch, both host bursts and
concurrent single calls through the C ABI and checks every output against
the oracle (see its header).  A heap / stack / global overflow, a use after
free or a leak in our host code aborts it; leaks the HIP / HSA runtimes keep
until exit are suppressed (tests/asan/lsan.supp).  Run once on the real
device count and once with three virtual devices, so the sharded paths
(one slice per device, persistent slice workers) run under ASan too.
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "asan", "host_asan")


@pytest.mark.gpu
@pytest.mark.parametrize("virtual", [None, "3"])
def test_host_code_under_asan(virtual):
    if not os.path.exists(EXE):
        pytest.skip("tests/asan/host_asan not built (make -C tests/asan)")
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:halt_on_error=1"
    env["LSAN_OPTIONS"] = "suppressions=" + os.path.join(HERE, "asan", "lsan.supp")
    env.pop("NET2_SHA2_VIRTUAL_DEVICES", None)
    if virtual:
        env["NET2_SHA2_VIRTUAL_DEVICES"] = virtual
    run = subprocess.run([EXE], capture_output=True, text=True, env=env, timeout=300)
    out = run.stdout + run.stderr
    print(out[-3000:])
    assert run.returncode == 0, out[-6000:]
    assert "host_asan ok" in run.stdout
    assert "AddressSanitizer" not in out and "LeakSanitizer" not in out
