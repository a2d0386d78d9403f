"""Key arenas: the engine's input layout (bytes + offsets, or fixed stride)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class Arena:
    """Host arena of n encoded keys; keeps the numpy buffers alive for the C call."""

    def __init__(self, keys: list[bytes]):
        n = len(keys)
        lens = np.fromiter((len(k) for k in keys), dtype=np.uint64, count=n)
        self.offsets = np.zeros(n + 1, dtype=np.uint64)
        if n:
            np.cumsum(lens, out=self.offsets[1:])
        blob = b"".join(keys)
        self.bytes = np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, np.uint8)
        self.n = n
        self.struct = L.RbxKeys(self.bytes.ctypes.data, self.offsets.ctypes.data, 0, n)

    @classmethod
    def fixed(cls, mat: np.ndarray) -> "Arena":
        a = cls.__new__(cls)
        mat = np.ascontiguousarray(mat, dtype=np.uint8)
        a.bytes = mat.reshape(-1) if mat.size else np.zeros(1, np.uint8)
        a.offsets = None
        a.n = mat.shape[0]
        a.struct = L.RbxKeys(a.bytes.ctypes.data, None, mat.shape[1], a.n)
        return a

    def ptr(self):
        return C.byref(self.struct)


class _OneKey:
    """add(T) / contains(T): one encoded key as an rbx_keys of stride len(key) over the bytes object itself
    (no numpy arena; the bytes object stays referenced for the call)."""

    __slots__ = ("key", "n", "struct")

    def __init__(self, key: bytes):
        self.key = key if type(key) is bytes else bytes(key)
        self.n = 1
        self.struct = L.RbxKeys(C.cast(C.c_char_p(self.key), C.c_void_p).value, None, len(self.key), 1)

    def ptr(self):
        return C.byref(self.struct)


def device_keys(data_ptr: int, n: int, stride: int = 0, offsets_ptr: int | None = None) -> L.RbxKeys:
    """rbx_keys over DEVICE memory (e.g. torch tensor data_ptr())."""
    return L.RbxKeys(data_ptr, offsets_ptr, stride, n)
