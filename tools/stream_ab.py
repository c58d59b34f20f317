#!/usr/bin/env python3
"""A/B of how bench steps are issued: one stream or two alternating streams,
with or without a HIP event pair around every launch.

A step is the same one-pass launch sequence bench.py times (device_step);
with two streams each stream has its own digest buffer and binning
workspace, so consecutive steps share only the (read-only) input batch and
the tail of one launch can overlap the head of the next.  Prints one line
per (config, mode, alternation): ms per step over `--steps` steps between
device synchronisations.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def run(name, mode, steps, warmup, dev, inp, outs, wss, streams):
    import torch
    nstr = 2 if mode.startswith("2") else 1
    events = mode.endswith("ev")
    fns = [bench.device_step(name, inp, outs[i], wss[i], streams[i])
           for i in range(nstr)]
    t = time.perf_counter()
    while time.perf_counter() - t < 0.3:
        for f in fns:
            f()
        torch.cuda.synchronize(dev)
    for k in range(warmup):
        fns[k % nstr]()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)] if events else None
    t0 = time.perf_counter()
    for k in range(steps):
        s = streams[k % nstr]
        if events:
            ev[k][0].record(s)
        fns[k % nstr]()
        if events:
            ev[k][1].record(s)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3 / steps
    kms = sum(a.elapsed_time(b) for a, b in ev) / steps if events else None
    return ms, kms


def main():
    import torch
    from ilias_net2_amd import batch
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4")
    ap.add_argument("--modes", default="1ev,1,2ev,2")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--alternations", type=int, default=3)
    ap.add_argument("--knob", default="NET2_KNOB",
                    help="environment variable an A/B build reads per launch "
                    "(the shipped library reads none; used with --values)")
    ap.add_argument("--values", default="",
                    help="comma list of values of --knob to A/B")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    for name in a.configs.split(","):
        cfg = bench.CONFIGS[name]
        inp = bench.make_inputs(cfg, dev, seed=2)
        n = inp["n"]
        dlen = bench.DLEN[cfg["alg"]]
        outs = [torch.empty((n, dlen), dtype=torch.uint8, device=dev) for _ in range(2)]
        wss = [batch.var_workspace(n, dev) if cfg["kind"] == "mixed" else None
               for _ in range(2)]
        streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
        occs = a.values.split(",") if a.values else [None]
        ref = None
        for occ in occs:      # every knob value gives the same digests
            if occ is not None:
                os.environ[a.knob] = occ
            bench.device_step(name, inp, outs[0], wss[0], streams[0])()
            torch.cuda.synchronize(dev)
            if ref is None:
                ref = outs[0].clone()
            print(f"{name} {a.knob}={occ} same_digests="
                  f"{bool(torch.equal(ref, outs[0]))}", flush=True)
        del ref
        for alt in range(a.alternations):
            for occ in occs:
                if occ is not None:
                    os.environ[a.knob] = occ
                for mode in a.modes.split(","):
                    ms, kms = run(name, mode, a.steps, a.warmup, dev, inp, outs,
                                  wss, streams)
                    print(f"{name} {a.knob}={occ} mode={mode:4s} alt={alt} "
                          f"ms_per_step={ms:.4f} "
                          f"event_ms={kms if kms is None else round(kms, 4)}",
                          flush=True)
        os.environ.pop(a.knob, None)
        from ilias_net2_amd import _lib
        torch.cuda.synchronize(dev)
        for k, w in enumerate(wss):     # did every binning launch bin?
            if w is not None:
                print(f"{name} workspace {k}: "
                      f"{_lib.workspace_stats(w.data_ptr(), w.numel() * 4)}", flush=True)
        del inp, outs, wss
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
