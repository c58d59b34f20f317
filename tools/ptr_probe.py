#!/usr/bin/env python3
"""Device mappings of host buffers (no kernel launch): hipPointerGetAttributes
and hipHostGetDevicePointer for a torch pinned buffer and for registered
(hipHostRegister) numpy memory, at the start and at an interior offset."""
import ctypes

import numpy as np
import torch

torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so.7")


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int),
                ("devicePointer", ctypes.c_void_p), ("hostPointer", ctypes.c_void_p),
                ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def show(name, p):
    a = Attr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    dp = ctypes.c_void_p()
    rc2 = hip.hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(p), 0)
    print(f"{name:28s} p={p:#x} attr rc={rc} type={a.type} dev={a.device} "
          f"devptr={a.devicePointer or 0:#x} hostptr={a.hostPointer or 0:#x} "
          f"flags={a.allocationFlags:#x} | getdevptr rc={rc2} dp={dp.value or 0:#x} "
          f"delta={(dp.value or 0) - p}", flush=True)
    # allocation range / buffer id (sha2_shim.cpp pinned_span)
    for nm, code in (("RANGE_START_ADDR", 11), ("RANGE_SIZE", 12), ("BUFFER_ID", 7)):
        v = ctypes.c_uint64(0)
        rc3 = hip.hipPointerGetAttribute(ctypes.byref(v), ctypes.c_int(code),
                                         ctypes.c_void_p(p))
        print(f"    {nm:16s} rc={rc3} v={v.value:#x}", flush=True)
    base = ctypes.c_void_p()
    size = ctypes.c_size_t()
    rc4 = hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(p))
    print(f"    hipMemGetAddressRange rc={rc4} base={base.value or 0:#x} size={size.value:#x}",
          flush=True)


t = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
show("torch pinned start", t.data_ptr())
show("torch pinned +13", t.data_ptr() + 13)
buf = np.zeros(1 << 21, dtype=np.uint8)
a0 = (buf.ctypes.data + 4095) & ~4095
cr = torch.cuda.cudart()
print("register rc", int(cr.cudaHostRegister(a0, 1 << 20, 0)), flush=True)
show("registered start", a0)
show("registered +13", a0 + 13)
show("registered +65536+13", a0 + 65536 + 13)
show("registered last byte", a0 + (1 << 20) - 1)
show("registered one past", a0 + (1 << 20))
print("unregister rc", int(cr.cudaHostUnregister(a0)), flush=True)
show("pageable", buf.ctypes.data)
# two pinned allocations back to back: is the second one's start the first's end?
u = torch.empty(4096, dtype=torch.uint8).pin_memory()
v = torch.empty(4096, dtype=torch.uint8).pin_memory()
print(f"adjacent pinned: u={u.data_ptr():#x} v={v.data_ptr():#x} "
      f"gap={v.data_ptr() - u.data_ptr()}", flush=True)
show("u last byte", u.data_ptr() + 4095)
show("v first byte", v.data_ptr())
