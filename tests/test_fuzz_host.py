"""CPU: libFuzzer targets under AddressSanitizer + UBSan for the host code
that parses bytes from the wire and for the oracle every GPU parity test
trusts (tests/fuzz/*.c).  Each test builds its target with the ROCm clang
(the only compiler here that carries libFuzzer) and runs a bounded, seeded
campaign; a crash, a sanitizer report or a failed check inside the target
fails the test with the fuzzer's output.

  wire_fuzz    net2x_signature_decode / _encode and the signed-carver header
               (include/net2/wire.h; types/signature.n2t:48-53,
               signed_carver_header.n2t:21-43): whatever decodes re-encodes
               to the bytes consumed; everything else is EINVAL.
  oracle_fuzz  the oracle's SHA-2 (one-shot, streamed in the input's split
               points) and HMAC against OpenSSL, and its packet decode /
               encode (types/packet.n2t:170-463) on raw and sealed datagrams.
"""
import os
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang"
# -fno-merge-all-constants -fdata-sections: with this clang, -fsanitize=fuzzer
# otherwise places the oracle's constant tables at unaligned addresses, which
# ASan reports as an ODR violation before the first input
FLAGS = ["-O1", "-g", "-std=c11", "-D_GNU_SOURCE",
         "-fsanitize=fuzzer,address,undefined", "-fno-sanitize-recover=undefined",
         "-fno-gpu-sanitize", "-Wno-unused-command-line-argument",   # host code only
         "-fno-merge-all-constants", "-fdata-sections"]

TARGETS = {
    "wire_fuzz": (["tests/fuzz/wire_fuzz.c", "ilias_net2_amd/csrc/host/wire.c",
                   "ilias_net2_amd/csrc/host/signature.c",
                   "ilias_net2_amd/csrc/host/sign.c"],
                  ["-Lilias_net2_amd", "-lnet2_sha2", "-lcrypto", "-lpthread",
                   f"-Wl,-rpath,{ROOT}/ilias_net2_amd"], 200000, 256),
    "oracle_fuzz": (["tests/fuzz/oracle_fuzz.c", "oracle/sha2_oracle.c"],
                    ["-lcrypto", "-lpthread"], 20000, 700),
}


def _field(b):
    """cxx_src/cp.cc:20-104: be32 length, bytes, zero pad to a multiple of 8."""
    return struct.pack(">I", len(b)) + b + b"\0" * (7 - (3 + len(b)) % 8)


# starting inputs that reach the success paths (the fuzzer mutates from here)
SEEDS = {
    "wire_fuzz": [_field(b"ecdsa") + _field(b"SHA512") + _field(bytes(range(37))),
                  _field(b"") + _field(b"") + _field(b"")],
    "oracle_fuzz": [bytes([2, 16, 1]) + bytes(range(256)) * 2,
                    bytes([0, 0, 0]) + b"abc"],
}


def _need_toolchain():
    if not os.path.exists(CLANG):
        pytest.skip("ROCm clang not present")
    if not os.path.exists(os.path.join(ROOT, "ilias_net2_amd", "libnet2_sha2.so")):
        pytest.skip("libnet2_sha2.so not built")


@pytest.mark.parametrize("name", sorted(TARGETS))
def test_fuzz_target(name, tmp_path):
    _need_toolchain()
    srcs, libs, runs, max_len = TARGETS[name]
    exe = tmp_path / name
    build = subprocess.run([CLANG, *FLAGS, "-o", str(exe),
                            *[os.path.join(ROOT, s) for s in srcs], *libs],
                           cwd=ROOT, capture_output=True, text=True)
    if build.returncode != 0 and "fuzzer" in build.stderr and "not found" in build.stderr:
        pytest.skip("libFuzzer runtime missing")
    assert build.returncode == 0, build.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    corpus = tmp_path / "corpus"
    corpus.mkdir()
    for k, seed in enumerate(SEEDS[name]):
        (corpus / f"seed{k}").write_bytes(seed)
    run = subprocess.run([str(exe), f"-runs={runs}", f"-max_len={max_len}",
                          "-seed=1", "-print_final_stats=1", str(corpus)],
                         cwd=tmp_path, capture_output=True, text=True, env=env,
                         timeout=600)
    out = run.stderr + run.stdout
    assert run.returncode == 0, out[-4000:]
    assert f"Done {runs} runs" in out, out[-2000:]
    assert not any(p.name.startswith(("crash-", "leak-", "timeout-"))
                   for p in tmp_path.iterdir())
    shutil.rmtree(tmp_path, ignore_errors=True)
