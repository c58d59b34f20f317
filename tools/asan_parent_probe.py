# Probe (tools/asan_hang_probe.sh): run tests/asan/host_asan as the child of a
# process that has (argv[1] == "torch") or has not initialised the GPU, output
# to argv[2]; PROBE_ASAN_OPTIONS overrides the ASan options.
import os, subprocess, sys, torch
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    torch.zeros(1, device="cuda")
env = dict(os.environ, ASAN_OPTIONS=os.environ.get("PROBE_ASAN_OPTIONS", "detect_leaks=1:abort_on_error=0:halt_on_error=1"),
           LSAN_OPTIONS="suppressions=" + os.path.abspath("tests/asan/lsan.supp"))
with open(sys.argv[2], "w") as f:
    r = subprocess.run(["./tests/asan/host_asan"], stdout=f, stderr=f, env=env, timeout=90)
print("rc", r.returncode)
