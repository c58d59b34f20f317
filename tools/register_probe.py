#!/usr/bin/env python3
"""Does a hipHostRegister record outlive hipHostUnregister + free?

Registers the first half of a page-aligned numpy buffer (as
tests/test_gpu_failures.py's half-registered test does), unregisters it,
frees the array, then allocates arrays of the same size until one lands at
the same address, and asks hipPointerGetAttributes what that address is now.
No kernel, no copy: attribute queries only.
"""
import ctypes
import gc

import numpy as np
import torch

torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so.7")


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int),
                ("devicePointer", ctypes.c_void_p), ("hostPointer", ctypes.c_void_p),
                ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def kind(p):
    a = Attr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    hip.hipGetLastError()
    return rc, a.type


cr = torch.cuda.cudart()
for size in (20000, 80000, 2_600_000, 40_000_000):
    buf = np.zeros(size + 8192, dtype=np.uint8)
    start = (buf.ctypes.data + 4095) & ~4095
    half = ((start + size // 2) & ~4095) - start
    assert int(cr.cudaHostRegister(start, half, 0)) == 0
    during = kind(start + 16)
    assert int(cr.cudaHostUnregister(start)) == 0
    after_unreg = kind(start + 16)
    base = buf.ctypes.data
    del buf
    gc.collect()
    hits = []
    keep = []
    for _ in range(50):
        b = np.zeros(size + 8192, dtype=np.uint8)
        keep.append(b)
        if b.ctypes.data <= start < b.ctypes.data + b.nbytes:
            hits.append(kind(start + 16))
            break
    print(f"size {size}: registered {half} B at {start:#x} (buffer {base:#x}); "
          f"during={during} after_unregister={after_unreg} "
          f"reallocated_same_range={bool(hits)} attr_now={hits[:1]}", flush=True)
    del keep
