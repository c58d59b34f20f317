#!/usr/bin/env python3
"""Per-chunk host timings (NET2_SHA2_DEBUG_TIMING=1, printed by the library
to stderr) of one RX and one TX host burst of 1 M MTU datagrams from pinned
memory, after a warm-up call each: where a call's time goes chunk by chunk.

  NET2_SHA2_DEBUG_TIMING=1 python tools/burst_debug_timing.py [n]
  REPS=20 [ORDER=rx-first] python tools/burst_debug_timing.py
                                     (call times only, back to back)
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ilias_net2_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    L = _lib.lib()
    rng = np.random.default_rng(11)
    lens = rng.choice(np.array([136, 584, 1500], dtype=np.uint32), n)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum())

    def pinned(shape, dt=torch.uint8):
        return torch.empty(shape, dtype=dt, pin_memory=True).numpy()
    data = pinned((total,))
    data[:] = rng.integers(0, 256, total, dtype=np.uint8)
    res, iv = pinned((n,)), pinned((n, 16))
    oseq, ofl = pinned((n,), torch.int32), pinned((n,), torch.int32)
    seq = np.arange(n, dtype=np.uint32)
    flags = np.full(n, 3, dtype=np.uint32)
    key = bytes(range(64))
    kb = ctypes.create_string_buffer(key, 64)
    keys = _lib.BurstRxKeys(6, ctypes.cast(kb, ctypes.c_void_p), 64, 1, None, 0, 0, 0, 0)
    p = lambda a: a.ctypes.data  # noqa: E731

    def tx():
        _lib.check(L.net2_packet_encode_burst_host(6, key, 64, 1, p(seq), p(flags),
                                                   p(data), p(offs), p(lens), n,
                                                   p(res), 1), "tx")

    def rx():
        _lib.check(L.net2_packet_decode_burst_host(ctypes.byref(keys), 16, p(data),
                                                   p(offs), p(lens), n, p(res), p(iv),
                                                   p(oseq), p(ofl), 1), "rx")
    reps = int(os.environ.get("REPS", "1"))
    seqs = [("tx", tx)] * reps + [("rx", rx)] * reps
    if os.environ.get("ORDER") == "rx-first":
        seqs = seqs[reps:] + seqs[:reps]
    def throttled():
        """The cgroup's CPU throttling counters (cgroup v2), if readable."""
        try:
            st = dict(ln.split() for ln in open("/sys/fs/cgroup/cpu.stat"))
            return f"nr_throttled {st.get('nr_throttled')} " \
                   f"throttled_usec {st.get('throttled_usec')} usage_usec {st.get('usage_usec')}"
        except (OSError, ValueError):
            return "cpu.stat n/a"
    def thread_cpu():
        """CPU seconds of this process's threads, by thread name."""
        tick = os.sysconf("SC_CLK_TCK")
        by = {}
        for tid in os.listdir("/proc/self/task"):
            try:
                name = open(f"/proc/self/task/{tid}/comm").read().strip()
                f = open(f"/proc/self/task/{tid}/stat").read().rsplit(")", 1)[1].split()
                by[name] = by.get(name, 0.0) + (int(f[11]) + int(f[12])) / tick
            except (OSError, ValueError, IndexError):
                pass
        return by

    def cpu_report(label, a, b, calls):
        rows = sorted(((b.get(k, 0.0) - a.get(k, 0.0), k) for k in b), reverse=True)
        txt = ", ".join(f"{k} {d * 1e3 / calls:.1f}" for d, k in rows if d > 0)
        print(f"-- CPU ms per call by thread, {label}: {txt}", file=sys.stderr)
    print("cpu.max:", open("/sys/fs/cgroup/cpu.max").read().strip()
          if os.path.exists("/sys/fs/cgroup/cpu.max") else "n/a", file=sys.stderr)
    prev, cur_kind, ncalls = None, None, 0
    for k, (name, fn) in enumerate([("tx", tx), ("rx", rx)] + seqs):
        if k >= 2 and name != cur_kind:
            now = thread_cpu()
            if prev is not None:
                cpu_report(cur_kind, prev, now, ncalls)
            prev, cur_kind, ncalls = now, name, 0
        t0 = time.perf_counter()
        fn()
        ncalls += 1
        print(f"== {name} {n} datagrams: {(time.perf_counter() - t0) * 1e3:.3f} ms  "
              f"[{throttled()}]", file=sys.stderr, flush=True)
    if prev is not None:
        cpu_report(cur_kind, prev, thread_cpu(), ncalls)


if __name__ == "__main__":
    main()
