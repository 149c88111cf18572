"""Loader for the in-tree native libraries.

* ``sketch_rnn_amd/_lib/libskrnn_host.so`` -- C++ host runtime (batch
  packer, ...), built with g++ by ``scripts/build_native.py``.
* ``sketch_rnn_amd/_lib/libskrnn_hip.so`` -- HIP kernels for gfx950, built
  with ``hipcc --offload-arch=gfx950``; exports a C ABI (``skr_*``) that
  takes raw device pointers and a ``hipStream_t``. It links the HIP runtime
  by soname, so when loaded after ``import torch`` it binds to the runtime
  PyTorch already mapped (one runtime per process).

Both are loaded with ``ctypes`` (no pybind / no torch headers). The HIP
library is required on GPU runs: :func:`require_hip` raises if it is absent.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib")
HOST_LIB = os.path.join(LIB_DIR, "libskrnn_host.so")
# SKR_HIP_LIB: load another build of the kernel library (A/B experiments,
# e.g. scripts/build_native.py --variant exact_act)
HIP_LIB = os.environ.get("SKR_HIP_LIB") or os.path.join(LIB_DIR, "libskrnn_hip.so")

_host = None
_hip = None

_c_f32p = ctypes.POINTER(ctypes.c_float)
_c_f64p = ctypes.POINTER(ctypes.c_double)
_c_i64p = ctypes.POINTER(ctypes.c_int64)


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


class HostLib:
    def __init__(self, lib: ctypes.CDLL):
        self.lib = lib
        lib.skr_pack_reference.restype = ctypes.c_int64
        lib.skr_pack_reference.argtypes = [_c_f32p, _c_i64p, ctypes.c_int64, _c_i64p, ctypes.c_int64,
                                           ctypes.c_int64, ctypes.POINTER(ctypes.c_int32), ctypes.c_int64,
                                           ctypes.c_int64, _c_f64p, _c_f32p]

    def pack_reference(self, flat: np.ndarray, offsets: np.ndarray, perm: np.ndarray, pointer: int,
                       finished: bool, batch: int, n: int, scales: np.ndarray, out: np.ndarray):
        assert flat.dtype == np.float32 and flat.flags.c_contiguous and flat.shape[1] == 4
        assert offsets.dtype == np.int64 and perm.dtype == np.int64
        assert scales.dtype == np.float64 and scales.shape == (batch, 2)
        assert out.dtype == np.float32 and out.shape == (batch, n, 5) and out.flags.c_contiguous
        fin = ctypes.c_int32(1 if finished else 0)
        ptr = self.lib.skr_pack_reference(_ptr(flat, _c_f32p), _ptr(offsets, _c_i64p), len(offsets) - 1,
                                          _ptr(perm, _c_i64p), len(perm), pointer, ctypes.byref(fin),
                                          batch, n, _ptr(scales, _c_f64p), _ptr(out, _c_f32p))
        if ptr < 0:
            raise RuntimeError("native packer failed (code %d)" % ptr)
        return int(ptr), bool(fin.value)


def host_lib() -> Optional[HostLib]:
    global _host
    if _host is None and os.path.exists(HOST_LIB):
        _host = HostLib(ctypes.CDLL(HOST_LIB))
    return _host


def hip_lib():
    """The HIP kernel library (``ctypes.CDLL``) or ``None`` if not built."""
    global _hip
    if _hip is None and os.path.exists(HIP_LIB):
        import torch  # noqa: F401  (map torch's HIP runtime first)
        from ..ops import _hipapi
        _hip = _hipapi.bind(ctypes.CDLL(HIP_LIB))
    return _hip


def require_hip():
    lib = hip_lib()
    if lib is None:
        raise RuntimeError("libskrnn_hip.so not found at %s: run `python scripts/build_native.py` "
                           "(or __graft_entry__.build()) before using the GPU path" % HIP_LIB)
    return lib


def hip_lib_stamp() -> dict:
    """Identity of the loaded HIP kernel library: its path, the content stamp
    scripts/build_native.py wrote beside it (sha256 of the sources, headers,
    flags and toolchain it was built from) and the file's own sha256 prefix."""
    import hashlib
    info = {"path": os.path.relpath(HIP_LIB, os.path.dirname(LIB_DIR)) if HIP_LIB.startswith(LIB_DIR) else HIP_LIB}
    try:
        with open(HIP_LIB + ".sha256") as f:
            info["source_stamp"] = f.read().strip()[:16]
    except OSError:
        info["source_stamp"] = None
    try:
        h = hashlib.sha256()
        with open(HIP_LIB, "rb") as f:
            for chunk in iter(lambda: f.read(1 << 20), b""):
                h.update(chunk)
        info["file_sha256"] = h.hexdigest()[:16]
    except OSError:
        info["file_sha256"] = None
    return info

