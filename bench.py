#!/usr/bin/env python3
"""Benchmark of the MI355X batched SHA-2 path (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): 1,048,576 x 1 KiB packets per
GPU, SHA-256, device-resident.  One step = one launch of the hot path over
the whole batch.  Multi-GPU: one process per GPU (torch.distributed.run),
each rank hashes its own shard -- packets are independent, so there is no
data-path collective; only the timing barrier and the max-over-ranks
reduction talk across ranks.

Prints ONE JSON line on rank 0.  --config selects another BASELINE config
for DESIGN.md numbers (c3 mixed, c4 SHA-512, e2e host-memory path).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SHA-256 digests/s over device-resident 1 KiB packets; HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters
# Vector-instruction issue peak: 256 CU x 4 SIMD, one wave64 VALU op per
# 2 cycles per SIMD (SIMD-32), 2.4 GHz max clock (MI355X_MICROARCH.md).
VALU_PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / 2

CONFIGS = {
    "c2": dict(alg=1, kind="fixed", n=1 << 20, length=1024,
               workload="1M x 1 KiB packets, SHA-256, device-resident (BASELINE configs[1])"),
    "c3": dict(alg=1, kind="mixed", n=1 << 20, length=None,
               workload="1M x mixed {64,512,1500} B packets, SHA-256, length-binned (configs[2])"),
    "c4": dict(alg=3, kind="fixed", n=1 << 20, length=1024,
               workload="1M x 1 KiB packets, SHA-512, device-resident (configs[3])"),
    # byte-aligned packet starts (lengths not multiples of 4): the A1 load
    # path of the variable-length kernel (not a BASELINE config)
    "c3_a1": dict(alg=1, kind="mixed", n=1 << 20, length=None, choice=[63, 511, 1499],
                  workload="1M x mixed {63,511,1499} B packets (byte-aligned starts), SHA-256, length-binned"),
    # the negotiated sighash (SHA-512) over variable-length payloads: the
    # signed-carver flow's shape (not a BASELINE config)
    "c3_512": dict(alg=3, kind="mixed", n=1 << 20, length=None,
                   workload="1M x mixed {64,512,1500} B packets, SHA-512, length-binned"),
    # SURVEY.md 8f rows, for DESIGN.md (not BASELINE configs)
    "hmac": dict(alg=4, kind="fixed", n=1 << 20, length=1024,
                 workload="1M x 1 KiB packets, HMAC-SHA256, device-resident (8f row 1)"),
    "hmac_mtu": dict(alg=4, kind="mixed", n=1 << 20, length=None,
                     workload="1M x mixed {64,512,1500} B datagrams, HMAC-SHA256, binned (8f row 1)"),
    # HMAC-SHA512 is what select_hash (conn_negotiator.c:110-131) picks when
    # every registry row is offered: the default per-datagram authenticator
    "hmac512": dict(alg=6, kind="fixed", n=1 << 20, length=1024,
                    workload="1M x 1 KiB packets, HMAC-SHA512, device-resident (8f row 1)"),
    "hmac512_mtu": dict(alg=6, kind="mixed", n=1 << 20, length=None,
                        workload="1M x mixed {64,512,1500} B datagrams, HMAC-SHA512, binned (8f row 1)"),
    # RX side of the datagram authenticator: each {64,512,1500} B datagram
    # is a 32-byte HMAC field || message (types/packet.n2t:226-257); one
    # result byte per datagram
    "hmac_verify_mtu": dict(alg=4, kind="dgram_verify", n=1 << 20, length=None,
                            workload="1M x mixed {64,512,1500} B datagrams, HMAC-SHA256 verify (hash field || message), binned (8f row 1, RX)"),
    "hmac512_verify_mtu": dict(alg=6, kind="dgram_verify", n=1 << 20, length=None,
                               workload="1M x mixed {64,512,1500} B datagrams, HMAC-SHA512 verify (hash field || message), binned (8f row 1, RX, the negotiated default)"),
    # the hash steps of net2_packet_decode / _encode for a burst under one
    # connection's keys (HMAC-SHA512 + AES-256-CBC IVs, every datagram
    # PH_SIGNED|PH_ENCRYPTED): wire sizes {136, 584, 1500} B = 8-byte header
    # + 64-byte HMAC field + {64, 512, 1428} B payload (8f row 3')
    "burst_rx": dict(alg=6, kind="burst_rx", n=1 << 20, length=None, ivlen=16,
                     workload="1M x {136,584,1500} B wire datagrams, net2_packet_decode_burst: header, HMAC-SHA512 verify, 16-B IVs (8f row 3', RX)"),
    "burst_tx": dict(alg=6, kind="burst_tx", n=1 << 20, length=None, ivlen=16,
                     workload="1M x {136,584,1500} B wire datagrams, net2_packet_encode_burst: header + HMAC-SHA512 field (8f row 3', TX)"),
    # the same burst under HMAC-SHA256 (a connection that negotiated it; the
    # SHA-256 kernels' RX mode, not a BASELINE config)
    "burst_rx256": dict(alg=4, kind="burst_rx", n=1 << 20, length=None, ivlen=16,
                        workload="1M x {136,584,1500} B wire datagrams, net2_packet_decode_burst: header, HMAC-SHA256 verify, 16-B IVs (8f row 3', RX)"),
    "ph_iv": dict(alg=1, kind="ph_iv", n=1 << 20, length=16,
                  workload="1M packet headers -> 16-byte IVs, net2_ph_to_iv_dev (8f row 3)"),
}
DLEN = {1: 32, 2: 48, 3: 64, 4: 32, 5: 48, 6: 64}
ALG_NAMES = {1: "SHA-256", 2: "SHA-384", 3: "SHA-512", 4: "HMAC-SHA256",
             5: "HMAC-SHA384", 6: "HMAC-SHA512"}
HMAC_KEY = bytes(range(64))
EVENT_EVERY = 4     # event pair around every 4th timed step (kernel duration)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def make_inputs(cfg, dev, seed):
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    n = cfg["n"]
    if cfg["kind"] == "fixed":
        data = torch.randint(0, 256, (n * cfg["length"],), dtype=torch.uint8,
                             device=dev, generator=g)
        return dict(data=data, n=n, payload=n * cfg["length"])
    if cfg["kind"] == "ph_iv":
        seq = torch.arange(n, dtype=torch.int32, device=dev)
        flags = torch.randint(0, 1 << 30, (n,), dtype=torch.int32, device=dev,
                              generator=g)
        return dict(seq=seq, flags=flags, n=n, payload=8 * n)
    burst = cfg["kind"].startswith("burst")
    choice = torch.tensor([136, 584, 1500] if burst else cfg.get("choice", [64, 512, 1500]),
                          dtype=torch.int64, device=dev)
    lens = choice[torch.randint(0, 3, (n,), device=dev, generator=g)]
    offs = torch.zeros(n, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)[:-1]
    total = int(lens.sum().item())
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev,
                         generator=g)
    r = dict(data=data, n=n, offs=offs, lens=lens.to(torch.int32), payload=total)
    if burst:
        r["seq"] = torch.arange(n, dtype=torch.int32, device=dev)
        r["flags"] = torch.full((n,), 3, dtype=torch.int32, device=dev)  # SIGNED|ENCRYPTED
        r["iv"] = torch.empty((n, cfg["ivlen"]), dtype=torch.uint8, device=dev)
        r["oseq"] = torch.empty(n, dtype=torch.int32, device=dev)
        r["oflags"] = torch.empty(n, dtype=torch.int32, device=dev)
    return r


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _smt_active():
    """SMT state of the host (SURVEY.md 8(d) asks for it), or None."""
    try:
        with open("/sys/devices/system/cpu/smt/active") as f:
            return f.read().strip() == "1"
    except OSError:
        return None


def _cpu_topology():
    """Physical cores and sockets from /proc/cpuinfo, cgroup CPU quota."""
    phys, cores_per = set(), None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys.add(line.split(":")[1].strip())
                elif line.startswith("cpu cores") and cores_per is None:
                    cores_per = int(line.split(":")[1])
    except OSError:
        pass
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                quota = f.read().strip()
            break
        except OSError:
            continue
    return {"physical_cores": (cores_per or 0) * max(len(phys), 1) or None,
            "sockets": len(phys) or None, "cgroup_cpu_quota": quota}


def _time_oracle(run, threads, reps=3):
    run(threads)  # warm-up (page faults, thread start)
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        run(threads)
        best = min(best, time.perf_counter() - t0)
    return best


SHA2C_RATIO = os.path.join(ROOT, "profiles", "round3", "sha2c_ratio.json")


def sha2c_ratio():
    """The port's speed over the reference's own src/sha2.c on identical
    batches, measured in the build container (tools/sha2c_ratio.sh; the
    reference tree is not on the GPU box): a labelled constant that turns
    the box's port figures into src/sha2.c figures."""
    try:
        with open(SHA2C_RATIO) as f:
            summ = json.load(f)["summary"]
    except (OSError, KeyError, ValueError):
        return None
    return {"port_over_sha2c": summ["port_batch_over_sha2c_geomean"],
            "range": [summ["min"], summ["max"]], "rows": summ["rows"],
            "source": "profiles/round3/sha2c_ratio.json (tools/sha2c_ratio.sh: "
                      "src/sha2.c built where it lies with include/net2/sha2.h, "
                      "C2/C3/C4 batches, rolled and unrolled, 1 and 8 threads, "
                      "build container; digests identical)"}


def cpu_baseline(cfg, light=False):
    """Oracle (clean-room C restatement of src/sha2.c, -O3) on the host
    cores of the GPU box: every usable host CPU (the headline value), the
    per-GPU share of 16 threads, and one thread.  light:
    the 16-thread share in both transform forms and one thread only (the
    C3 / C4 lines of extra_configs, a few seconds each)."""
    from oracle import oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth
    affinity = len(os.sched_getaffinity(0))
    share = min(16, affinity)
    allc = min(256, affinity)          # oracle_sha2_batch caps at 256 threads
    alg = cfg["alg"]
    n = cfg["n"]
    if cfg["kind"] == "fixed":
        data = synth.fixed_batch(2, n, cfg["length"])
        run = lambda t, m=n, u=False: oracle.batch(  # noqa: E731
            alg, data, stride=cfg["length"], length=cfg["length"], n=m,
            nthreads=t, unrolled=u)
    else:
        lens = synth.mixed_lengths(3, n)
        data, offs = synth.packed(4, lens)
        run = lambda t, m=n, u=False: oracle.batch(  # noqa: E731
            alg, data, offsets=offs[:m], lens=lens[:m], nthreads=t, unrolled=u)
    # both transforms of src/sha2.c: rolled (:374-445, the default build)
    # and unrolled (:316-370, SHA2_UNROLL_TRANSFORM)
    t_share = _time_oracle(run, share)
    t_all = _time_oracle(run, allc, reps=5) if not light else float("inf")
    t_share_u = _time_oracle(lambda t: run(t, n, True), share)
    # one thread, on the first n/16 packets (same shape)
    n1 = max(1, n // 16)
    t0 = time.perf_counter()
    run(1, n1)
    single = n1 / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    run(1, n1, True)
    single_u = n1 / (time.perf_counter() - t0)
    ratio = sha2c_ratio()
    what = cfg["workload"].split(" packets")[0]
    form_ref = {"rolled": "src/sha2.c:374-445", "unrolled": "src/sha2.c:316-370"}
    if light:
        best_t, best_form = min((t_share, "rolled"), (t_share_u, "unrolled"))
        return {"value": n / best_t, "unit": "digests/s", "cores": share,
                "kind": "port",
                "sample": (f"the full {what} packet batch from host memory, "
                           f"oracle/sha2_oracle.c (-O3, {best_form} transform like "
                           f"{form_ref[best_form]}) on {share} pthreads (the per-GPU "
                           f"share), best of 3 after a warm-up"),
                "rolled_value": n / t_share, "unrolled_value": n / t_share_u,
                "single_thread_value": max(single, single_u),
                "reference_sha2c": (dict(ratio, value=round(n / best_t / ratio["port_over_sha2c"], 1))
                                    if ratio else None)}
    # Context, not the baseline the north star names: the same batch through
    # OpenSSL's SHA*_Init/Update/Final, the calls the reference's C++ layer
    # makes (cxx_src/hash-openssl.cc:25-131; SHA-NI on this host's EPYC).
    if cfg["kind"] == "fixed":
        ossl = lambda t, m=n: oracle.openssl_batch(  # noqa: E731
            alg, data, stride=cfg["length"], length=cfg["length"], n=m, nthreads=t)
    else:
        ossl = lambda t, m=n: oracle.openssl_batch(  # noqa: E731
            alg, data, offsets=offs[:m], lens=lens[:m], nthreads=t)
    t_ossl = _time_oracle(ossl, share)
    ossl(1, n1)
    t0 = time.perf_counter()
    ossl(1, n1)
    single_ossl = n1 / (time.perf_counter() - t0)
    topo = _cpu_topology()
    # The headline is the best measured rate.  On the GPU boxes of this pool
    # the process sees every CPU of the node (affinity) but its cgroup
    # grants 16 CPUs of time (cpu.max "1600000 100000"), so a thread per
    # host CPU runs no faster than 16; the whole-node rate is then
    # extrapolated, and labelled so, from the one-thread rate.
    best_t, best_threads, best_form = min((t_share, share, "rolled"),
                                          (t_all, allc, "rolled"),
                                          (t_share_u, share, "unrolled"))
    phys = topo.get("physical_cores")
    return {"value": n / best_t, "unit": "digests/s", "cores": best_threads,
            "kind": "port",
            "sample": (f"the full {what} packet batch from host memory, "
                       f"oracle/sha2_oracle.c (-O3, {best_form} transform like "
                       f"{form_ref[best_form]}) on {best_threads} pthreads, best "
                       f"of 3-5 after a warm-up (fastest of: the 16-thread "
                       f"per-GPU share, one thread per usable host CPU, the "
                       f"unrolled transform on the 16-thread share)"),
            "per_gpu_share": {"value": n / t_share, "threads": share},
            "all_host_cpus": {"value": n / t_all, "threads": allc,
                              "note": "one thread per CPU in the affinity mask; "
                                      "bounded by cgroup_cpu_quota when one is set"},
            "unrolled_transform": {"value": n / t_share_u, "threads": share,
                                   "single_thread_value": single_u,
                                   "form": "SHA2_UNROLL_TRANSFORM, " + form_ref["unrolled"]},
            "whole_node_extrapolated": (
                {"value": max(single, single_u) * phys,
                 "basis": f"best single_thread_value x {phys} physical cores "
                          "(an estimate, not a measurement; SMT not credited)"}
                if phys else None),
            "single_thread_value": single,
            # the reference's own src/sha2.c is not on the GPU box: its rate
            # here is the port's over the ratio measured in the build container
            "reference_sha2c": (dict(ratio, value=round(n / best_t / ratio["port_over_sha2c"], 1))
                                if ratio else None),
            "openssl_context": {
                "value": n / t_ossl, "threads": share,
                "single_thread_value": single_ossl,
                "note": "not the src/sha2.c baseline: OpenSSL's SHA*_Init/"
                        "Update/Final as the reference's C++ layer calls them "
                        "(cxx_src/hash-openssl.cc:25-131), system libcrypto, "
                        "its own SHA-NI / AVX2 transform; oracle/openssl_batch.c"},
            "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "affinity_cpus": affinity, "smt_active": _smt_active(), **topo}


def gpu_info(dev):
    """Name, host and shader clock of the GPU (the box-to-box spread of the
    pool is larger than run-to-run noise)."""
    import socket
    import torch
    p = torch.cuda.get_device_properties(dev)
    bus = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    return {"name": p.name, "arch": p.gcnArchName, "cus": p.multi_processor_count,
            "pci": bus, "host": socket.gethostname(),
            "sclk_mhz": read_sclk(bus)}


def read_sclk(bus):
    """(max, current) shader clock in MHz from the amdgpu DPM table."""
    try:
        with open(f"/sys/bus/pci/devices/{bus}/pp_dpm_sclk") as f:
            rows = f.read().split("\n")
    except OSError:
        return None
    mhz, cur = [], None
    for r in rows:
        parts = r.replace(":", " ").split()
        for tok in parts:
            if tok.lower().endswith("mhz"):
                v = int(tok[:-3])
                mhz.append(v)
                if "*" in r:
                    cur = v
    return {"max": max(mhz) if mhz else None, "current": cur}


def library_build_id():
    """The kernel build the loaded libnet2_sha2.so was compiled from."""
    from ilias_net2_amd import _lib
    return _lib.lib().net2_sha2_build_id().decode()


def load_pmc(config_name):
    """Per-launch HBM traffic / VALU counts from the committed rocprofv3 PMC
    summary (profiles/pmc_<config>.json, written by tools/pmc_summary.py),
    with whether it was measured on the kernel build that is loaded now
    (its kernel_build_id stamp)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config_name}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        pmc = json.load(f)
    return pmc, pmc.get("kernel_build_id") == library_build_id()


def load_isa_mix(config_name):
    """Instruction mix of the config kernel's block loop, priced with the
    probed issue costs (profiles/isa_mix.json, written by tools/isa_mix.py);
    None unless it was taken from the kernel build that is loaded now."""
    path = os.path.join(ROOT, "profiles", "isa_mix.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        mix = json.load(f)
    if mix.get("kernel_build_id") != library_build_id():
        return None
    return mix["configs"].get(config_name)


def device_step(name, inp, out, ws_buf, stream, unbinned=False, kind=None):
    """One step of a device-resident config: one pass of the hot path over
    the whole batch (one launch, plus the binning launches of the variable
    layout).  kind overrides the config's (the untimed encode of an RX
    burst, under the config's own algorithm)."""
    from ilias_net2_amd import batch, _lib
    cfg = dict(CONFIGS[name])
    if kind is not None:
        cfg["kind"] = kind
    L = _lib.lib()
    n, alg = inp["n"], cfg["alg"]
    kbuf = HMAC_KEY[:DLEN[alg]] if alg >= 4 else b""
    if cfg["kind"] == "burst_rx":
        return lambda: _lib.check(L.net2_packet_decode_burst(
            alg, kbuf, len(kbuf), 1, cfg["ivlen"], inp["data"].data_ptr(),
            inp["offs"].data_ptr(), inp["lens"].data_ptr(), n, out.data_ptr(),
            inp["iv"].data_ptr(), inp["oseq"].data_ptr(), inp["oflags"].data_ptr(),
            ws_buf.data_ptr(), ws_buf.numel(), stream.cuda_stream))
    if cfg["kind"] == "burst_tx":
        return lambda: _lib.check(L.net2_packet_encode_burst(
            alg, kbuf, len(kbuf), 1, inp["seq"].data_ptr(), inp["flags"].data_ptr(),
            inp["data"].data_ptr(), inp["offs"].data_ptr(), inp["lens"].data_ptr(),
            n, out.data_ptr(), ws_buf.data_ptr(), ws_buf.numel(), stream.cuda_stream))
    if cfg["kind"] == "dgram_verify":
        return lambda: _lib.check(L.net2_hmac_verify_dev(
            alg, kbuf, len(kbuf), inp["data"].data_ptr(),
            inp["offs"].data_ptr(), inp["lens"].data_ptr(), n,
            out.data_ptr(), ws_buf.data_ptr(), ws_buf.numel() * 4,
            stream.cuda_stream))
    if cfg["kind"] == "ph_iv":
        return lambda: _lib.check(L.net2_ph_to_iv_dev(
            inp["seq"].data_ptr(), inp["flags"].data_ptr(), n, cfg["length"],
            out.data_ptr(), stream.cuda_stream))
    if alg >= 4:
        mixed = cfg["kind"] == "mixed"
        return lambda: _lib.check(L.net2_hmac_dev(
            alg, kbuf, len(kbuf), inp["data"].data_ptr(),
            inp["offs"].data_ptr() if mixed else None,
            inp["lens"].data_ptr() if mixed else None,
            cfg["length"] or 0, cfg["length"] or 0, n, out.data_ptr(),
            ws_buf.data_ptr() if mixed and not unbinned else None,
            ws_buf.numel() * 4 if mixed else 0, stream.cuda_stream))
    if cfg["kind"] == "fixed":
        return lambda: batch.digest_fixed(alg, inp["data"], cfg["length"],
                                          cfg["length"], n, out=out,
                                          stream=stream)
    return lambda: batch.digest_var(alg, inp["data"], inp["offs"], inp["lens"],
                                    out=out, workspace=ws_buf,
                                    binned=not unbinned, stream=stream)


def time_device_config(name, dev, steps, warmup, prewarm_ms, ws=1, rank=0,
                       dist_backend="nccl", unbinned=False, clock_probe=None):
    """Untimed clock ramp and warmup, then exactly `steps` steps between
    barriers + synchronize; the dominant kernel's duration from HIP events
    on the launch stream.  Returns the measurements (max over ranks)."""
    import torch
    import torch.distributed as dist
    from ilias_net2_amd import batch, _lib
    cfg = CONFIGS[name]
    inp = make_inputs(cfg, dev, seed=2 + rank)
    n, alg = inp["n"], cfg["alg"]
    burst = cfg["kind"].startswith("burst")
    dlen = cfg["length"] if cfg["kind"] == "ph_iv" else \
        1 if cfg["kind"] == "dgram_verify" or burst else DLEN[alg]
    out = torch.empty((n, dlen), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    ws_buf = batch.var_workspace(n, dev) if cfg["kind"] in ("mixed", "dgram_verify") else None
    if burst:
        ws_buf = torch.empty(_lib.lib().net2_packet_burst_workspace(n),
                             dtype=torch.uint8, device=dev)
    if cfg["kind"] == "burst_rx":
        # encode once (untimed), so every datagram verifies and gets its IV
        device_step(name, inp, out, ws_buf, stream, kind="burst_tx")()
        torch.cuda.synchronize(dev)
        assert int((out != 0).sum()) == 0, "burst encode failed"
    if cfg["kind"] == "dgram_verify":
        # sign once (untimed) so every datagram verifies
        batch.hmac_sign_dev(alg, HMAC_KEY[:DLEN[alg]], inp["data"], inp["offs"],
                            inp["lens"], workspace=ws_buf)
    step = device_step(name, inp, out, ws_buf, stream, unbinned)
    # Clock ramp: repeat the step (untimed) for prewarm_ms of wall time.
    t_pw = time.perf_counter()
    while (time.perf_counter() - t_pw) * 1e3 < prewarm_ms:
        step()
        torch.cuda.synchronize(dev)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    # HIP events on the stream the kernels are launched on, around every
    # EVENT_EVERY-th step: an event pair adds ~7 us of queue time to the step
    # it brackets (profiles/round2/stream_events_ab.txt), so bracketing every
    # step would bill that to the throughput; the sampled launches give the
    # kernel duration.
    sampled = [k % EVENT_EVERY == 0 for k in range(steps)]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(sum(sampled))]
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    j = 0
    for k in range(steps):
        if sampled[k]:
            ev[j][0].record(stream)
            step()
            ev[j][1].record(stream)
            j += 1
        else:
            step()
    enqueue_ms = (time.perf_counter() - t0) * 1e3
    # shader clock while the queued steps run, sampled every ~2 ms by a
    # helper thread (a sysfs read can take a millisecond: kept off the
    # thread whose synchronize ends the timed region)
    samples, stop = [], threading.Event()

    def sample():
        while not stop.is_set():
            c = clock_probe()
            if not c:
                return
            samples.append(c)
            stop.wait(0.002)
    sampler = threading.Thread(target=sample, daemon=True) if clock_probe else None
    if sampler:
        sampler.start()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if sampler:
        stop.set()
        sampler.join()
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    local_ms = elapsed * 1e3 / steps    # this rank's own, before the max
    if burst:   # every datagram of the synthetic burst is well-formed
        assert int((out != 0).sum()) == 0, f"{name}: datagrams not OK"

    if ws > 1:
        t = torch.tensor([elapsed, launch_ms], dtype=torch.float64,
                         device=dev if dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, launch_ms = float(t[0]), float(t[1])
    # algorithmic bytes: payload read + digests written (+ 12 B/packet of
    # offsets and lengths for the variable layout), per launch
    per_launch = inp["payload"] + n * dlen + \
        (12 * n if cfg["kind"] in ("mixed", "dgram_verify") or burst else 0)
    if cfg["kind"] == "burst_rx":     # + decoded header and IV out
        per_launch += n * (8 + cfg["ivlen"])
    elif cfg["kind"] == "burst_tx":   # + header in; header + field written
        per_launch += n * (8 + 8 + DLEN[alg])
    res = {"n": n, "dlen": dlen, "payload": inp["payload"], "elapsed": elapsed,
           "ms_per_step": elapsed * 1e3 / steps, "launch_ms": launch_ms,
           "ms_per_step_local": local_ms,
           "host_enqueue_ms": enqueue_ms,
           "event_pairs": len(ev),
           "per_launch_bytes": per_launch,
           "sclk_during_mhz": (round(sum(samples) / len(samples)) if samples else None),
           "sclk_samples": len(samples), "sclk_min_mhz": min(samples) if samples else None}
    del inp, out, ws_buf
    torch.cuda.empty_cache()
    return res


def rooflines(name, launch_ms, per_launch, sclk_mhz=None):
    """HBM roofline of the dominant kernel (algorithmic bytes over the
    event-timed launch, PMC traffic from profiles/pmc_<config>.json) and the
    VALU issue figures that bind these kernels."""
    achieved = per_launch / (launch_ms / 1e3) / 1e9
    pmc, fresh = load_pmc(name)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel_ms": round(launch_ms, 4),
            "algorithmic_bytes_per_launch": per_launch}
    if pmc and not fresh:
        # counters of another kernel build: not this build's traffic
        roof["traffic_note"] = (
            "profiles/pmc_%s.json was measured on kernel build %s, the loaded "
            "library is %s: counters not reported" % (
                name, pmc.get("kernel_build_id"), library_build_id()))
        pmc = None
    pmc_mhz = (pmc.get("clock_ghz_under_pmc") or 0) * 1e3 if pmc else 0
    if pmc and sclk_mhz and pmc_mhz and abs(pmc_mhz / sclk_mhz - 1) > 0.03:
        # counters taken at another shader clock than this line's timed
        # steps (a throttled or other box): per-launch counts would still
        # hold, but the cycle figures priced with them would not
        roof["traffic_note"] = (
            "profiles/pmc_%s.json was measured at %.0f MHz, this line's timed "
            "steps at %.0f MHz (> 3 %% apart): counters not joined" % (
                name, pmc_mhz, sclk_mhz))
        pmc = None
    box_mhz = ((pmc or {}).get("trace_box") or {}).get("sclk_mhz_during_timed_steps")
    if pmc and sclk_mhz and box_mhz and abs(box_mhz / sclk_mhz - 1) > 0.03:
        # the kernel trace committed beside the counters was taken on a box
        # that timed this config at another clock: its average duration
        # would not be this line's
        roof["traffic_note"] = (
            "profiles/pmc_%s.json's trace box timed this config at %d MHz, "
            "this line's timed steps ran at %.0f MHz (> 3 %% apart): counters "
            "not joined" % (name, box_mhz, sclk_mhz))
        pmc = None
    if pmc:
        roof["counters_clock_mhz"] = round(pmc_mhz) if pmc_mhz else None
        roof["counters_box"] = pmc.get("trace_box")
        roof["trace_kernel_ms"] = round(pmc["trace_avg_ns"] / 1e6, 4) \
            if pmc.get("trace_avg_ns") else None
    if pmc:
        roof["traffic"] = pmc.get("hbm_bytes_per_launch")
        roof["traffic_build_id"] = pmc.get("kernel_build_id")
    if pmc and pmc.get("hbm_bytes_per_launch"):
        roof["traffic_over_algorithmic"] = round(pmc["hbm_bytes_per_launch"] / per_launch, 3)
    valu = None
    if pmc and pmc.get("valu_wave_instr_per_launch"):
        instr = pmc["valu_wave_instr_per_launch"]
        rate = instr / (launch_ms / 1e3)
        # cycles at this line's own clock (the counted instructions do not
        # depend on it; the launch time does)
        clk = (sclk_mhz / 1e3 if sclk_mhz else None) or \
            pmc.get("clock_ghz_under_pmc") or 2.4
        valu = {"bound": "valu", "achieved": round(rate / 1e12, 4),
                "peak": round(VALU_PEAK_WAVE_INSTR / 1e12, 4),
                "unit": "T wave64-VALU-instr/s",
                "frac": round(rate / VALU_PEAK_WAVE_INSTR, 4),
                # SIMD cycles between VALU issues, averaged over the launch:
                # 2.0 = the nominal SIMD-32 rate, reached only by full-rate
                # ops in a pure stream; v_alignbit/v_add3/v_perm are
                # half-rate (4.2), and a stream mixing the two classes issues
                # every instruction at ~4
                "simd_cycles_per_valu_instr": round(clk * 1e9 * (launch_ms / 1e3) * 1024 / instr, 3),
                "clock_ghz": round(clk, 3),
                "instr_per_launch": instr,
                "source": "rocprofv3 SQ_INSTS_VALU / GRBM_GUI_ACTIVE, profiles/pmc_%s.json" % name}
        mix = load_isa_mix(name)
        if mix and mix.get("mean_issue_cycles_per_valu_instr"):
            # Issue floor: every VALU instruction of the launch priced at the
            # measured issue cost of a mixed half/full-rate stream
            # (tools/isa_mix.py, probe cycles at 2.4 GHz like the probe).
            m = mix["mean_issue_cycles_per_valu_instr"]
            floor_ms = instr / 1024 * m / 2.4e9 * 1e3
            valu["issue_floor"] = {
                "mean_cycles_per_valu_instr": m,
                "floor_ms": round(floor_ms, 4),
                "frac": round(floor_ms / launch_ms, 4),
                **({"floor_ms_at_timed_sclk": round(floor_ms * 2400.0 / sclk_mhz, 4),
                    "frac_at_timed_sclk": round(floor_ms * 2400.0 / sclk_mhz / launch_ms, 4),
                    "timed_sclk_mhz": sclk_mhz} if sclk_mhz else {}),
                "source": "profiles/isa_mix.json (mixed-stream model) x profiles/round1/valu_bank_seq_probe.json (cost)"}
            step = pmc.get("step_valu_wave_instr")
            if step and step > instr and sclk_mhz:
                # the same floor over the VALU work of every launch of the
                # step (binning, the burst final kernel's IV derivation),
                # priced at the same cost: what the step could take
                sfl = step / 1024 * m / (sclk_mhz * 1e6) * 1e3
                valu["issue_floor"]["step"] = {
                    "instr_per_step": step,
                    "kernels": sorted(pmc.get("step_kernels_valu", {})),
                    "floor_ms_at_timed_sclk": round(sfl, 4),
                    "frac_at_timed_sclk": round(sfl / launch_ms, 4)}
    return roof, valu


def metric_of(name):
    cfg = CONFIGS[name]
    alg = cfg["alg"]
    if name == "c2":
        return METRIC
    return (("SHA-256 IVs/s, " if cfg["kind"] == "ph_iv" else
             f"{ALG_NAMES[alg]} datagrams verified/s, " if cfg["kind"] == "dgram_verify" else
             "datagrams decoded/s, " if cfg["kind"] == "burst_rx" else
             "datagrams encoded/s, " if cfg["kind"] == "burst_tx" else
             f"{ALG_NAMES[alg]} digests/s, ") + cfg["workload"])


def unit_of(name):
    kind = CONFIGS[name]["kind"]
    return "datagrams/s" if kind in ("dgram_verify", "burst_rx", "burst_tx") else "IVs/s" if kind == "ph_iv" else "digests/s"


def pci_numa_node(pci):
    try:
        with open(f"/sys/bus/pci/devices/{pci}/numa_node") as f:
            return int(f.read())
    except (OSError, ValueError, TypeError):
        return None


def rank_record(rank, gpu, ms_per_step):
    """What each rank contributes to an N>1 line: where it ran and its own
    time per step (before the max over ranks)."""
    return {"rank": rank, "host": gpu.get("host"), "pci": gpu.get("pci"),
            "numa_node": pci_numa_node(gpu.get("pci")),
            "ms_per_step": round(ms_per_step, 4)}


def gather_ranks(rec, ws):
    """Every rank's record, in rank order, on every rank."""
    if ws == 1:
        return [rec]
    import torch.distributed as dist
    out = [None] * ws
    dist.all_gather_object(out, rec)
    return out


def scale_fields(ranks, backend):
    """Fields of an N>1 line that say on which devices its ranks ran.  Under
    RCCL ("nccl", the driver's scaling runs) two ranks on one GPU would make
    the line's n_gpus a lie: that is an error, raised on every rank (all
    hold the same records).  A gloo rehearsal that shares a device is
    labelled so instead."""
    keys = [(r["host"], r["pci"]) for r in ranks]
    distinct = len(set(keys))
    shared = distinct < len(ranks)
    if shared and backend == "nccl":
        dup = sorted({k for k in keys if keys.count(k) > 1})
        raise SystemExit(f"bench.py: {len(ranks)} ranks but {distinct} distinct "
                         f"GPUs (shared: {dup}); one process per GPU is required")
    ms = [r["ms_per_step"] for r in ranks]
    return {"distinct_devices": distinct,
            "device_sharing": (f"shared device: {len(ranks)} ranks on {distinct} GPU(s), "
                               "a rehearsal, not an N-GPU measurement") if shared
            else "one GPU per rank",
            "ms_per_step_ranks": {"min": min(ms), "max": max(ms)},
            "ranks": ranks}


def devices_label(ws, distinct):
    return f"{ws} GPU(s)" if distinct == ws else \
        f"{ws} ranks on {distinct} shared GPU(s)"


def cpu_baseline_after_gpu(cfg, rank, ws, fn=None):
    """cpu_baseline at any N, on rank 0 after every GPU step of the line is
    done, so the 1/2/4/8-GPU lines each carry a same-box CPU figure (north
    star).  The other ranks wait on the rendezvous store (a blocking socket
    wait: no rank spins a CPU while rank 0 times the host)."""
    import torch.distributed as dist
    res = (fn or cpu_baseline)(cfg) if rank == 0 else None
    if ws > 1:
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("net2_bench_cpu_baseline_done", "1")
        else:
            store.wait(["net2_bench_cpu_baseline_done"])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--prewarm-ms", type=float, default=500.0,
                    help="untimed launches before the warmup steps so the GPU "
                         "reaches its steady-state clock (a cold MI355X runs "
                         "the first ~50 launches ~15%% slower)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS) + ["e2e", "c1"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="c2 at N=1: skip the extra BASELINE configs (C1, C3, C4, "
                         "end to end) that otherwise ride in the same line")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--unbinned", action="store_true",
                    help="c3: hash in submission order (ablation)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from ilias_net2_amd import _lib

    ws, rank, local = dist_env()
    # One process per GPU.  --dist-backend gloo with more ranks than GPUs
    # (device = local rank mod device count) rehearses the N>1 path on a
    # 1-GPU box; the driver's multi-GPU runs use RCCL ("nccl").
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", (local % ndev) if ws > 1 else 0)
    torch.cuda.set_device(dev)
    if ws > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    if _lib.device_count() < 1:
        raise SystemExit("no gfx950 device visible to libnet2_sha2.so")

    if args.config == "e2e":
        return run_e2e(args, ws, rank, dev)
    if args.config == "c1":
        print(json.dumps(run_c1()), flush=True)
        return None

    gpu = gpu_info(dev)
    probe = lambda: (read_sclk(gpu["pci"]) or {}).get("current")  # noqa: E731
    name = args.config
    cfg = CONFIGS[name]
    r = time_device_config(name, dev, args.steps, args.warmup, args.prewarm_ms,
                           ws, rank, args.dist_backend, args.unbinned, probe)
    value = r["n"] * ws / (r["ms_per_step"] / 1e3)
    roof, valu = rooflines(name, r["launch_ms"], r["per_launch_bytes"],
                           r["sclk_during_mhz"])
    roof["event_pairs"] = r["event_pairs"]
    alg = cfg["alg"]
    line = {
        "metric": metric_of(name),
        "value": round(value, 1),
        "unit": unit_of(name),
        "n_gpus": ws,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(r["ms_per_step"], 4), "higher_is_better": True,
        "prewarm_ms": args.prewarm_ms,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64" if alg in (2, 3, 5, 6) else "u32",
        "data": "synthetic: uniform random bytes (torch.randint, seed 2+rank), resident in HBM before timing",
        "config": {"workload": cfg["workload"] + (" [unbinned]" if args.unbinned else ""),
                   "packets_per_gpu": r["n"],
                   "alg": ALG_NAMES[alg].replace("-", "") if alg <= 3 else ALG_NAMES[alg],
                   "payload_bytes_per_gpu": r["payload"],
                   "parallelism": f"{ws} independent shards, no collective"},
        "roofline": roof,
    }
    if valu:
        line["roofline_valu"] = valu
    gpu["sclk_mhz_during_timed_steps"] = r["sclk_during_mhz"]
    line["gpu"] = gpu
    # host time to queue the timed steps (rank 0's): near the whole timed
    # region means the launches, not the GPU, set the pace
    line["host_enqueue_ms"] = round(r["host_enqueue_ms"], 3)
    ranks = gather_ranks(rank_record(rank, gpu, r["ms_per_step_local"]), ws)
    if ws > 1:
        sf = scale_fields(ranks, args.dist_backend)
        line.update(sf)
        line["config"]["parallelism"] = (
            f"{ws} independent shards, no collective; " + sf["device_sharing"])
    if name == "c2" and not args.no_extras:
        line["extra_configs"] = extra_configs(
            args, dev, probe, ws, rank,
            label=devices_label(ws, line.get("distinct_devices", ws)))
    if not args.no_cpu_baseline and name in ("c2", "c3", "c4"):
        cb = cpu_baseline_after_gpu(cfg, rank, ws)
        if rank == 0:
            line["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(finalize_line(line)), flush=True)
    if ws > 1:
        dist.destroy_process_group()
    return None


# Strings kept where they are when a line is finalized; any other string
# over NOTE_MIN characters moves to the line's "notes" (finalize_line).
KEEP_PROSE = {("metric",), ("unit",), ("data",), ("config", "workload"),
              ("config", "parallelism"), ("cpu_baseline", "sample"),
              ("cpu_baseline", "unit"), ("cpu_baseline", "kind")}
NOTE_MIN = 60


def _hoist(obj, path, notes):
    for k in list(obj):
        v, p = obj[k], path + (k,)
        if isinstance(v, dict):
            _hoist(v, p, notes)
        elif isinstance(v, str) and len(v) > NOTE_MIN and p not in KEEP_PROSE:
            notes[".".join(p)] = v
            del obj[k]


def _brief(r):
    """The numbers of one config for the line's closing summary."""
    if not isinstance(r, dict):
        return None
    out = {k: r[k] for k in ("value", "ms_per_step") if k in r}
    roof = r.get("roofline") or {}
    for k, kk in (("kernel_ms", "kernel_ms"), ("frac", "frac"),
                  ("traffic_over_algorithmic", "traffic_x")):
        if roof.get(k) is not None:
            out[kk] = roof[k]
    if isinstance(r.get("pageable"), dict):
        out["pageable_value"] = r["pageable"].get("value")
    cb = r.get("cpu_baseline")
    if isinstance(cb, dict) and cb.get("value"):
        out["cpu_value"] = round(cb["value"], 1)
    return out


def finalize_line(line):
    """The printed form of a line: long prose moved into one "notes" object
    near the front, and every config's numbers repeated in a short
    "summary" that closes the line, so a reader of only its last ~2 KB (the
    driver's record keeps a tail) still has C2, C3, C4 and the end-to-end
    rates."""
    notes = {}
    body = dict(line)
    for k in list(body):
        if isinstance(body[k], dict):
            _hoist(body[k], (k,), notes)
    front = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
             "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")
    out = {k: body.pop(k) for k in front if k in body}
    if notes:
        out["notes"] = notes
    out.update(body)
    summary = {"line": _brief(line)}
    for k, r in (line.get("extra_configs") or {}).items():
        b = _brief(r)
        if k == "c1" and isinstance(r, dict):
            st = r.get("stages", {})
            b = {s: st[s].get("ms") for s in ("gpu_digest_sha512", "cpu_digest_sha512_1core",
                                               "sc_hash_tick") if s in st}
        if k == "burst_small" and isinstance(r, dict):
            b = {kk: r[kk] for kk in ("rx", "tx") if kk in r}
        if b:
            summary[k] = b
    out["summary"] = summary
    return out


def extra_configs(args, dev, probe, ws=1, rank=0, label=None):
    """The other BASELINE.json configs, timed in the same invocation: at
    N=1, C3 (mixed lengths, binned) and C4 (SHA-512) device-resident with
    their rooflines, C1 (4096 x 1 KiB signed payloads) and the end-to-end
    host-memory rate; at N>1 the end-to-end rate over all ranks -- C5,
    1 M x 1 KiB per GPU from pinned host memory through every GPU at once
    (8 M at N=8), the max over ranks of the per-step time."""
    out = {}
    if ws > 1:
        out["e2e"] = e2e_rate(steps=10, warmup=3, ws=ws, dev=dev,
                              dist_backend=args.dist_backend, label=label)
        # the per-datagram path from host memory on every GPU at once
        out["burst_rx_e2e"] = burst_e2e_rate("rx", steps=6, warmup=2, ws=ws, dev=dev,
                                             dist_backend=args.dist_backend,
                                             label=label)
        return out
    for name in ("c3", "c4"):
        r = time_device_config(name, dev, args.steps, min(args.warmup, 10),
                               200.0, clock_probe=probe)
        roof, valu = rooflines(name, r["launch_ms"], r["per_launch_bytes"],
                           r["sclk_during_mhz"])
        roof["event_pairs"] = r["event_pairs"]
        out[name] = {"metric": metric_of(name), "value": round(r["n"] / (r["ms_per_step"] / 1e3), 1),
                     "unit": unit_of(name), "steps": args.steps,
                     "ms_per_step": round(r["ms_per_step"], 4),
                     "workload": CONFIGS[name]["workload"],
                     "sclk_mhz_during_timed_steps": r["sclk_during_mhz"],
                     "roofline": roof}
        if valu:
            out[name]["roofline_valu"] = valu
        if rank == 0 and not args.no_cpu_baseline:
            out[name]["cpu_baseline"] = cpu_baseline(CONFIGS[name], light=True)
    out["e2e"] = e2e_rate(steps=10, warmup=3)
    # the per-datagram path from host memory (north_star: "starts and ends
    # in host memory"), pinned buffers; the pageable rate beside it
    for kind in ("rx", "tx"):
        r = burst_e2e_rate(kind)
        pg = burst_e2e_rate(kind, steps=4, warmup=1, memory="pageable")
        r["pageable"] = {k: pg[k] for k in ("value", "ms_per_step", "h2d_GBps")}
        out[f"burst_{kind}_e2e"] = r
    out["burst_small"] = burst_small_latency()
    out["c1"] = run_c1()
    return out


def burst_small_latency(sizes=(64, 1024, 4096), budget_s=0.3):
    """The integration's operating point (a receive loop
    hands over whatever the socket holds, NET2_BURST 4,096): median time of
    one net2_packet_decode_burst_host / _encode_burst_host call of 64 /
    1,024 / 4,096 {136, 584, 1500}-byte HMAC-SHA512 datagrams with 16-byte
    IVs from pinned host memory, one GPU, after two warm-up calls; every
    call's codes checked (DESIGN.md §6.4 has the whole table and the CPU
    beside it)."""
    import ctypes
    import statistics
    import numpy as np
    import torch
    from ilias_net2_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(11)
    nmax = max(sizes)
    lens_all = rng.choice(np.array([136, 584, 1500], dtype=np.uint32), nmax)
    key = HMAC_KEY[:64]
    kb = ctypes.create_string_buffer(key, 64)
    keys = _lib.BurstRxKeys(6, ctypes.cast(kb, ctypes.c_void_p), 64, 1, None, 0, 0, 0, 0)

    def pinned(shape, dt=torch.uint8):
        return torch.empty(shape, dtype=dt, pin_memory=True).numpy()
    p = lambda a: a.ctypes.data  # noqa: E731
    out = {"unit": "us per call (median)", "memory": "pinned",
           "workload": "HMAC-SHA512 + 16-byte IVs, {136, 584, 1500} B datagrams"}
    for kind in ("rx", "tx"):
        row = {}
        for n in sizes:
            lens = lens_all[:n].copy()
            offs = np.zeros(n, dtype=np.uint64)
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            data = pinned((int(lens.sum()),))
            data[:] = rng.integers(0, 256, data.size, dtype=np.uint8)
            res, iv = pinned((n,)), pinned((n, 16))
            oseq, ofl = pinned((n,), torch.int32), pinned((n,), torch.int32)
            seq = np.arange(n, dtype=np.uint32)
            flags = np.full(n, 3, dtype=np.uint32)

            def tx():
                _lib.check(L.net2_packet_encode_burst_host(
                    6, key, 64, 1, p(seq), p(flags), p(data), p(offs), p(lens), n,
                    p(res), 1), "net2_packet_encode_burst_host")

            def rx():
                _lib.check(L.net2_packet_decode_burst_host(
                    ctypes.byref(keys), 16, p(data), p(offs), p(lens), n, p(res), p(iv),
                    p(oseq), p(ofl), 1), "net2_packet_decode_burst_host")
            tx()                                # sealed once, then timed
            fn = rx if kind == "rx" else tx
            fn()
            fn()
            ts, t_all = [], time.perf_counter()
            while len(ts) < 400 and (time.perf_counter() - t_all < budget_s or len(ts) < 20):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            assert int((res != 0).sum()) == 0, f"burst_small {kind} {n}: not OK"
            row[str(n)] = round(statistics.median(ts) * 1e6, 1)
        out[kind] = row
    return out


def _parse_cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def gpu_local_cpus(dev):
    """CPUs of the NUMA node the GPU's PCIe link hangs off (sysfs), within
    this process's affinity; None when unknown."""
    import torch
    try:
        p = torch.cuda.get_device_properties(dev)
        bus = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            node = int(f.read())
        if node < 0:
            return None
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _parse_cpulist(f.read()) & os.sched_getaffinity(0)
        return cpus or None
    except (OSError, ValueError):
        return None


def e2e_rate(steps, warmup, n=1 << 20, length=1024, ws=1, dev=None,
             dist_backend="nccl", label=None):
    """C5's shape: 1 M x 1 KiB per GPU from pinned host memory -> the GPU ->
    digests back to pinned host memory, through net2_sha2_batch (each rank
    on its own GPU, max_devices 1); timed between barriers, max over ranks."""
    import torch
    import torch.distributed as dist
    from ilias_net2_amd import _lib
    # host buffers on the GPU's NUMA node (first touch by a thread running
    # there), as a NUMA-aware caller would place them; affinity restored after
    local = gpu_local_cpus(dev if dev is not None else torch.device("cuda", 0)) \
        if os.environ.get("NET2_BENCH_NUMA", "1") != "0" else None
    saved = os.sched_getaffinity(0)
    if local:
        os.sched_setaffinity(0, local)
    try:
        return _e2e_timed(steps, warmup, n, length, ws, dev, dist_backend,
                          numa=bool(local), label=label or f"{ws} GPU(s)")
    finally:
        os.sched_setaffinity(0, saved)


def _e2e_timed(steps, warmup, n, length, ws, dev, dist_backend, numa,
               label):
    import torch
    import torch.distributed as dist
    from ilias_net2_amd import _lib
    host = torch.randint(0, 256, (n * length,), dtype=torch.uint8).pin_memory()
    outp = torch.empty((n, 32), dtype=torch.uint8).pin_memory()
    L = _lib.lib()

    def step():
        _lib.check(L.net2_sha2_batch(1, host.data_ptr(), None, None, length,
                                     length, n, outp.data_ptr(), 1))
    for _ in range(warmup):
        step()
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if ws > 1:
        dist.barrier()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    ms_local = ms
    if ws > 1:
        t = torch.tensor([ms], dtype=torch.float64,
                         device=dev if dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t[0])
        t = torch.tensor([ms_local], dtype=torch.float64,
                         device=dev if dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ms_min = float(t[0])
    del host, outp
    return {"metric": "SHA-256 digests/s, 1 KiB packets from pinned host memory, "
                      f"end to end (H2D, kernel, digests stored to host memory), {label}",
            **({"ms_per_step_ranks": {"min": round(ms_min, 3), "max": round(ms, 3)}}
               if ws > 1 else {}),
            "value": round(n * ws / (ms / 1e3), 1), "unit": "digests/s", "steps": steps,
            "n_gpus": ws, "ms_per_step": round(ms, 3),
            "workload": f"{ws} x 1M x 1 KiB, host -> GPU -> host via net2_sha2_batch, "
                        "one rank per GPU (BASELINE configs[4] at N=8)",
            "h2d_GBps_per_gpu": round(n * length / (ms / 1e3) / 1e9, 2),
            "host_buffers_numa_local": numa}


def burst_e2e_rate(kind, steps=8, warmup=2, n=1 << 20, memory="pinned", ws=1,
                   dev=None, dist_backend="nccl", label="1 GPU"):
    """The burst configs end to end from host memory (VERDICT round 4 item
    1): 1 M wire datagrams of {136, 584, 1500} B (8-byte header, 64-byte
    HMAC-SHA512 field, payload; every one PH_SIGNED|PH_ENCRYPTED) in host
    memory -> net2_packet_decode_burst_host (RX: codes, headers and 16-byte
    IVs back to host memory) or net2_packet_encode_burst_host (TX: header
    and HMAC field sealed into the caller's buffer) on this process's GPU
    (max_devices 1).  The datagrams are sealed once, untimed, before the RX
    steps.  At N>1 every rank does the same on its own GPU at once (timed
    between barriers, max over ranks; value = all ranks' datagrams)."""
    import numpy as np
    import torch
    from ilias_net2_amd import _lib
    import ctypes
    L = _lib.lib()
    rng = np.random.default_rng(7)
    lens = rng.choice(np.array([136, 584, 1500], dtype=np.uint32), n)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum())
    seq = np.arange(n, dtype=np.uint32)
    flags = np.full(n, 3, dtype=np.uint32)
    key = HMAC_KEY[:64]

    def host(shape, dt):
        if memory == "pinned":
            t = torch.empty(shape, dtype={np.uint8: torch.uint8,
                                          np.uint32: torch.int32}[dt], pin_memory=True)
            return t.numpy().view(dt)
        return np.empty(shape, dtype=dt)
    data = host((total,), np.uint8)
    data[:] = rng.integers(0, 256, total, dtype=np.uint8)
    res = host((n,), np.uint8)
    p = lambda a: a.ctypes.data  # noqa: E731

    def tx():
        _lib.check(L.net2_packet_encode_burst_host(
            6, key, 64, 1, p(seq), p(flags), p(data), p(offs), p(lens), n,
            p(res), 1), "net2_packet_encode_burst_host")
    iv = host((n, 16), np.uint8)
    oseq, ofl = host((n,), np.uint32), host((n,), np.uint32)
    kb = ctypes.create_string_buffer(key, 64)
    keys = _lib.BurstRxKeys(6, ctypes.cast(kb, ctypes.c_void_p), 64, 1, None, 0, 0, 0, 0)

    def rx():
        _lib.check(L.net2_packet_decode_burst_host(
            ctypes.byref(keys), 16, p(data), p(offs), p(lens), n, p(res), p(iv),
            p(oseq), p(ofl), 1), "net2_packet_decode_burst_host")
    tx()
    assert int((res != 0).sum()) == 0, "burst seal failed"
    step = rx if kind == "rx" else tx
    for _ in range(warmup):
        step()
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if ws > 1:
        dist.barrier()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    if ws > 1:
        t = torch.tensor([ms], dtype=torch.float64,
                         device=dev if dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t[0])
    assert int((res != 0).sum()) == 0, f"burst {kind}: datagrams not OK"
    out_bytes = n * (1 + 16 + 8) if kind == "rx" else n * (1 + 8 + 64)
    r = {"metric": ("datagrams decoded/s" if kind == "rx" else "datagrams encoded/s") +
                   f", 1M x {{136,584,1500}} B wire datagrams from {memory} host memory, "
                   "end to end (pack, H2D, HMAC-SHA512" +
                   (" verify + 16-B IVs" if kind == "rx" else " seal") +
                   f", results to host memory), {label}",
         "value": round(n * ws / (ms / 1e3), 1), "unit": "datagrams/s", "steps": steps,
         "n_gpus": ws,
         "ms_per_step": round(ms, 3),
         "workload": f"net2_packet_{'decode' if kind == 'rx' else 'encode'}_burst_host, "
                     f"{memory} datagram buffer and result arrays, max_devices 1",
         "h2d_GBps" if ws == 1 else "h2d_GBps_per_gpu": round(total / (ms / 1e3) / 1e9, 2),
         "host_bytes_per_step": {"datagrams_in": total, "results_out": out_bytes}}
    del data, res, iv, oseq, ofl
    return r


def run_c1():
    """BASELINE configs[0] shape: 4096 x 1 KiB payloads through the signed-
    payload flow with test/sign.c's P-521 key (tools/bench_sign.py): GPU
    digests from host memory, the oracle's digests on one core (the
    reference's per-payload loop), and the batched signature create /
    validate (ECDSA on host threads)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_sign
    return bench_sign.measure()


def run_e2e(args, ws, rank, dev):
    """Config 5 shape: host memory -> pinned H2D -> kernel -> digests to host,
    through net2_sha2_batch on this rank's device (PCIe-inclusive rate)."""
    import torch
    import torch.distributed as dist
    gpu = gpu_info(dev)
    sf = None
    if ws > 1:
        sf = scale_fields(gather_ranks(rank_record(rank, gpu, 0.0), ws),
                          args.dist_backend)
    t0 = time.perf_counter()
    r = e2e_rate(args.steps, args.warmup, ws=ws, dev=dev,
                 dist_backend=args.dist_backend,
                 label=devices_label(ws, sf["distinct_devices"] if sf else ws))
    el = time.perf_counter() - t0
    if sf:
        r.update({"distinct_devices": sf["distinct_devices"],
                  "device_sharing": sf["device_sharing"],
                  "ranks": [dict(x, ms_per_step=None) for x in sf["ranks"]]})
    r["gpu"] = gpu
    r.update({"n_gpus": ws, "warmup": args.warmup, "higher_is_better": True,
              "scaling": "weak", "vs_baseline": None, "dtype": "u32",
              "data": "synthetic random bytes in pinned host memory",
              "wall_s": round(el, 3)})
    if rank == 0:
        print(json.dumps(r), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
