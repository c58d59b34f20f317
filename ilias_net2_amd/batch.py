"""Batched digests over device-resident or host packets (torch / numpy glue).

PyTorch is plumbing here: it owns device memory and streams; the digests come
from the HIP kernels behind ``net2_sha2_dev_fixed`` / ``net2_sha2_dev_var`` /
``net2_sha2_batch`` (include/net2/sha2_batch.h).  The batched entry is what
``net2_signature_create`` / ``_validate`` (types/signature.n2t:92,147) and
``net2_signctx_fingerprint`` (src/sign.c:298-307) reduce to when many payloads
are hashed at once.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from ._lib import DIGEST_LEN, check


def _need(t, dtype, what: str):
    """Device tensors are passed as raw pointers: check what the C ABI
    assumes (dtype, contiguity, a GPU device) before handing them over."""
    if t.dtype != dtype:
        raise TypeError(f"{what} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{what} must be contiguous")
    if t.device.type != "cuda":
        raise ValueError(f"{what} must live on the GPU")


def _stream_ptr(stream) -> Optional[int]:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _launch_stream(stream, device):
    """The torch stream a launch goes to: ``stream`` (a torch stream or a raw
    hipStream_t), default torch's current stream on ``device``.

    Temporaries (binning workspace, outputs allocated here) are allocated
    under this stream, so torch's caching allocator hands their memory out
    again only in this stream's order -- never while the kernel that uses
    them may still be running."""
    import torch
    if stream is None:
        return torch.cuda.current_stream(device)
    if isinstance(stream, int):
        return torch.cuda.ExternalStream(stream, device=device)
    return stream


def _check_data(data, stride: int, length: int, n: int):
    if n and data.numel() < (n - 1) * stride + length:
        raise ValueError("data tensor too small for n packets")


def _check_out(out, n: int, per: int):
    import torch
    _need(out, torch.uint8, "out")
    if out.numel() < n * per:
        raise ValueError("out too small")


def digest_fixed(alg: int, data, stride: int, length: int, n: int, out=None,
                 stream=None):
    """Digests of n packets data[i*stride : i*stride+length] (uint8 CUDA tensor).

    Returns an (n, hashlen) uint8 tensor on the same device.  Asynchronous on
    ``stream`` (default: torch's current stream)."""
    import torch
    dl = DIGEST_LEN[alg]
    _need(data, torch.uint8, "data")
    s = _launch_stream(stream, data.device)
    if out is None:
        with torch.cuda.stream(s):
            out = torch.empty((n, dl), dtype=torch.uint8, device=data.device)
    _check_out(out, n, dl)
    _check_data(data, stride, length, n)
    rc = _lib.lib().net2_sha2_dev_fixed(alg, data.data_ptr(), stride, length,
                                        n, out.data_ptr(), s.cuda_stream)
    check(rc, "net2_sha2_dev_fixed")
    return out


def var_workspace(n: int, device, stream=None):
    """Binning scratch for n packets, allocated and prepared
    (net2_sha2_workspace_init) in ``stream``'s order."""
    import torch
    nbytes = _lib.lib().net2_sha2_dev_var_workspace(n)
    s = _launch_stream(stream, device)
    with torch.cuda.stream(s):
        ws = torch.empty(((nbytes + 3) // 4,), dtype=torch.int32,
                         device=device)
    check(_lib.lib().net2_sha2_workspace_init(ws.data_ptr(), ws.numel() * 4,
                                              s.cuda_stream),
          "net2_sha2_workspace_init")
    return ws


def _workspace(n: int, device, s, workspace=None):
    """(pointer, bytes) of a caller's workspace, or of a temporary one
    allocated in stream s's order (freed on return, reused only by work
    ordered after this launch on s)."""
    if workspace is None:
        workspace = var_workspace(n, device, s)
    return workspace, workspace.data_ptr(), workspace.numel() * 4


def digest_var(alg: int, data, offsets, lens, out=None, workspace=None,
               binned: bool = True, stream=None):
    """Digests of packets data[offsets[i] : offsets[i]+lens[i]].

    data: uint8 CUDA tensor; offsets: int64 CUDA tensor; lens: int32 CUDA
    tensor.  binned=True sorts by block count on the device first.
    Asynchronous on ``stream`` (default: torch's current stream)."""
    import torch
    n = int(offsets.numel())
    dl = DIGEST_LEN[alg]
    _need(data, torch.uint8, "data")
    _need(offsets, torch.int64, "offsets")
    _need(lens, torch.int32, "lens")
    if lens.numel() != n:
        raise ValueError("offsets and lens differ in length")
    s = _launch_stream(stream, data.device)
    if out is None:
        with torch.cuda.stream(s):
            out = torch.empty((n, dl), dtype=torch.uint8, device=data.device)
    _check_out(out, n, dl)
    ws_ptr, ws_bytes = None, 0
    if binned and n:
        workspace, ws_ptr, ws_bytes = _workspace(n, data.device, s, workspace)
    rc = _lib.lib().net2_sha2_dev_var(alg, data.data_ptr(), offsets.data_ptr(),
                                      lens.data_ptr(), n, out.data_ptr(),
                                      ws_ptr, ws_bytes, s.cuda_stream)
    check(rc, "net2_sha2_dev_var")
    return out


def _np_ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def digest_host(alg: int, data: np.ndarray, offsets: Optional[np.ndarray] = None,
                lens: Optional[np.ndarray] = None, stride: int = 0,
                length: int = 0, n: Optional[int] = None,
                max_devices: int = 0) -> np.ndarray:
    """End-to-end batch from host memory (numpy) -> host digests (numpy)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = len(offsets)
    elif n is None:
        n = (len(data) // stride) if stride else 0
    out = np.empty((n, DIGEST_LEN[alg]), dtype=np.uint8)
    rc = _lib.lib().net2_sha2_batch(alg, _np_ptr(data), _np_ptr(offsets),
                                    _np_ptr(lens), stride, length, n,
                                    _np_ptr(out), max_devices)
    check(rc, "net2_sha2_batch")
    return out


def hmac_dev(alg: int, key: bytes, data, stride: int = 0, length: int = 0,
             n: Optional[int] = None, offsets=None, lens=None, out=None,
             binned: bool = True, stream=None, workspace=None):
    """Batched HMAC (registry rows 4..6) of device-resident packets under one
    key: fixed layout (stride/length/n) or variable layout (offsets/lens).
    Asynchronous on ``stream`` (default: torch's current stream); the key is
    copied into the launch's arguments, so it need not outlive the call."""
    import torch
    dl = DIGEST_LEN[alg]
    _need(data, torch.uint8, "data")
    if offsets is not None:
        _need(offsets, torch.int64, "offsets")
        _need(lens, torch.int32, "lens")
        n = int(offsets.numel())
        if lens.numel() != n:
            raise ValueError("offsets and lens differ in length")
    else:
        if n is None:
            raise ValueError("fixed layout needs n")
        _check_data(data, stride, length, n)
    s = _launch_stream(stream, data.device)
    if out is None:
        with torch.cuda.stream(s):
            out = torch.empty((n, dl), dtype=torch.uint8, device=data.device)
    _check_out(out, n, dl)
    kb = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    ws_ptr, ws_bytes = None, 0
    if offsets is not None and binned and n:
        workspace, ws_ptr, ws_bytes = _workspace(n, data.device, s, workspace)
    rc = _lib.lib().net2_hmac_dev(
        alg, kb, len(key), data.data_ptr(),
        None if offsets is None else offsets.data_ptr(),
        None if lens is None else lens.data_ptr(), stride, length, n,
        out.data_ptr(), ws_ptr, ws_bytes, s.cuda_stream)
    check(rc, "net2_hmac_dev")
    return out


def _dgram_args(key, data, offsets, lens):
    import torch
    _need(data, torch.uint8, "data")
    _need(offsets, torch.int64, "offsets")
    _need(lens, torch.int32, "lens")
    n = int(offsets.numel())
    if lens.numel() != n:
        raise ValueError("offsets and lens differ in length")
    kb = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    return n, kb


def hmac_sign_dev(alg: int, key: bytes, data, offsets, lens,
                  binned: bool = True, stream=None, workspace=None):
    """TX side of the per-datagram authenticator (types/packet.n2t:410-427):
    datagram i = data[offsets[i] : offsets[i] + lens[i]] is hash field ||
    message; the first hashlen bytes receive HMAC(key, message), in place.
    Asynchronous on ``stream``."""
    n, kb = _dgram_args(key, data, offsets, lens)
    s = _launch_stream(stream, data.device)
    ws_ptr, ws_bytes = None, 0
    if binned and n:
        workspace, ws_ptr, ws_bytes = _workspace(n, data.device, s, workspace)
    rc = _lib.lib().net2_hmac_sign_dev(
        alg, kb, len(key), data.data_ptr(), offsets.data_ptr(),
        lens.data_ptr(), n, ws_ptr, ws_bytes, s.cuda_stream)
    check(rc, "net2_hmac_sign_dev")
    return data


def hmac_verify_dev(alg: int, key: bytes, data, offsets, lens,
                    binned: bool = True, stream=None, out=None,
                    workspace=None):
    """RX side (types/packet.n2t:226-257): uint8 per datagram, 0 if its hash
    field equals HMAC(key, message), 1 if not, 2 if shorter than hashlen.
    Asynchronous on ``stream``."""
    import torch
    n, kb = _dgram_args(key, data, offsets, lens)
    s = _launch_stream(stream, data.device)
    if out is None:
        with torch.cuda.stream(s):
            out = torch.empty((n,), dtype=torch.uint8, device=data.device)
    _check_out(out, n, 1)
    ws_ptr, ws_bytes = None, 0
    if binned and n:
        workspace, ws_ptr, ws_bytes = _workspace(n, data.device, s, workspace)
    rc = _lib.lib().net2_hmac_verify_dev(
        alg, kb, len(key), data.data_ptr(), offsets.data_ptr(),
        lens.data_ptr(), n, out.data_ptr(), ws_ptr, ws_bytes, s.cuda_stream)
    check(rc, "net2_hmac_verify_dev")
    return out
