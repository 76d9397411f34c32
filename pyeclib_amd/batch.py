"""Batched, device-resident entry points (the ecamd_* half of the C ABI).

Objects and fragments stay in HBM; only per-object erasure bitmasks cross
from the host.  Buffers are anything exposing ``data_ptr()`` (torch tensors)
or raw integer device addresses, laid out as documented in
include/erasurecode_amd.h.  PyTorch is plumbing here (allocation, streams);
it never touches the payload arithmetic.
"""
from __future__ import annotations

import ctypes
from typing import Any, Sequence

from . import _native

HEADER = _native.HEADER_SIZE


def blocksize(k: int, obj_len: int, w: int = 16) -> int:
    """Payload bytes per fragment: the object padded to a multiple of
    k * w/8 bytes, split k ways (liberasurecode get_aligned_data_size; w = 16
    for rs_vand, 8 for the ISA-L codes)."""
    mult = k * (w // 8)
    return (obj_len + mult - 1) // mult * mult // k


def frag_stride(bs: int, align: int = 128) -> int:
    """Fragment slot size: header + payload (rounded to 16 B), rounded up to
    `align` bytes.  With 128 and fragments starting PAYLOAD_SKEW bytes into a
    128-B-aligned buffer, every payload starts on a 128-B cache line."""
    return (HEADER + (bs + 15) // 16 * 16 + align - 1) // align * align


# Fragment buffers start this many bytes past a 128-B boundary so that the
# payload (after the 80-byte header) is line-aligned: 48 + 80 = 128.
PAYLOAD_SKEW = 48


def stripe_buffer(n_obj: int, k: int, m: int, bs: int, device: Any = None) -> Any:
    """(n_obj, k+m, frag_stride) uint8 torch view whose payloads are 128-B aligned."""
    import torch
    fs = frag_stride(bs)
    flat = torch.zeros(n_obj * (k + m) * fs + 128, dtype=torch.uint8, device=device)
    base = flat.data_ptr() % 128
    off = (PAYLOAD_SKEW - base) % 128
    return flat[off:off + n_obj * (k + m) * fs].view(n_obj, k + m, fs)


def _ptr(x: Any) -> int:
    return int(x.data_ptr()) if hasattr(x, "data_ptr") else int(x)


def _stride0(x: Any, default: int) -> int:
    """Byte stride between objects of a (n_obj, ...) uint8 tensor."""
    return int(x.stride(0)) if hasattr(x, "stride") else default


def _stream(stream: Any) -> int | None:
    if stream is None:
        try:
            import torch
            return torch.cuda.current_stream().cuda_stream
        except Exception:
            return None
    return int(getattr(stream, "cuda_stream", stream))


# ec_type -> (backend id, field bits)
_CODES = {"amd_rs_vand": (11, 16), "liberasurecode_rs_vand": (6, 16),
          "isa_l_rs_vand": (4, 8), "isa_l_rs_cauchy": (7, 8)}


class BatchCodec:
    """One (k, m) instance of a GPU ec_type driving the batch kernels."""

    def __init__(self, k: int, m: int, inline_crc32: bool = False,
                 ec_type: str = "amd_rs_vand"):
        if ec_type not in _CODES:
            raise ValueError(f"{ec_type} has no GPU batch path")
        backend, self.w = _CODES[ec_type]
        self.k, self.m, self.ec_type = k, m, ec_type
        self.handle = _native.init(k, m, backend, m, 1 if inline_crc32 else 0, 0, 0, 0)

    def blocksize(self, obj_len: int) -> int:
        return blocksize(self.k, obj_len, self.w)

    def _check(self, ret: int, fn: str) -> None:
        if ret < 0:
            _native.raise_error(ret, fn)

    @staticmethod
    def _check_rows(fn: str, x: Any, rows: int | None = None) -> None:
        """A (n_obj, rows, stride) or (n_obj, stride) uint8 tensor must be
        packed the way the C side walks it: bytes contiguous, and -- for
        per-object groups of `rows` fragments -- each object's group at
        rows * stride(1) (the C API takes only the fragment stride, so a
        strided view such as stripes[:, :k] would be read as the wrong bytes)."""
        if x is None or not hasattr(x, "stride"):
            return
        dims = x.dim() if hasattr(x, "dim") else len(x.shape)
        if int(x.stride(dims - 1)) != 1:
            _native.raise_error(-_native.EINVALIDPARAMS, fn)
        if rows is not None:
            if dims != 3 or int(x.shape[1]) != rows or \
                    (int(x.shape[0]) > 1 and int(x.stride(0)) != rows * int(x.stride(1))):
                _native.raise_error(-_native.EINVALIDPARAMS, fn)

    @staticmethod
    def _check_count(fn: str, n_obj: int, *arrays: Any) -> None:
        """n_obj per-object entries must fit every tensor they index (the C
        entry points trust the caller's sizes)."""
        for a in arrays:
            if a is not None and hasattr(a, "shape") and n_obj > int(a.shape[0]):
                _native.raise_error(-_native.EINVALIDPARAMS, fn)

    def encode(self, objs: Any, obj_len: int, parity: Any, data: Any = None,
               frag_stride: int | None = None, stream: Any = None) -> None:
        """objs: (n_obj, obj_stride) uint8; parity: (n_obj, m, frag_stride)
        (a view into a (n_obj, k+m, frag_stride) stripe buffer works);
        data: optional (n_obj, k, frag_stride) view for materialised data
        fragments."""
        n_obj = int(objs.shape[0])
        self._check_count("ecamd_encode_batch", n_obj, parity, data)
        for x in (objs, parity, data):
            self._check_rows("ecamd_encode_batch", x)
        fs = frag_stride if frag_stride is not None else int(parity.stride(1))
        ret = _native.lib.ecamd_encode_batch(
            self.handle.desc, _ptr(objs), _stride0(objs, obj_len), obj_len, n_obj,
            _ptr(parity), _ptr(data) if data is not None else None, fs,
            _stride0(parity, self.m * fs), _stream(stream))
        self._check(ret, "ecamd_encode_batch")

    def decode(self, frags: Any, obj_len: int, avail_masks: Sequence[int], out: Any,
               stream: Any = None) -> None:
        """frags: (n_obj, k+m, frag_stride) stripes; out: (n_obj, obj_stride)."""
        n_obj = len(avail_masks)
        self._check_count("ecamd_decode_batch", n_obj, frags, out)
        for x in (frags, out):
            self._check_rows("ecamd_decode_batch", x)
        masks = (ctypes.c_uint32 * n_obj)(*avail_masks)
        fs = int(frags.stride(1))
        ret = _native.lib.ecamd_decode_batch(
            self.handle.desc, _ptr(frags), fs, _stride0(frags, (self.k + self.m) * fs), obj_len,
            n_obj, masks, _ptr(out), _stride0(out, obj_len), _stream(stream))
        self._check(ret, "ecamd_decode_batch")

    def reconstruct(self, frags: Any, obj_len: int, avail_masks: Sequence[int],
                    dest: Sequence[int], out: Any, stream: Any = None) -> None:
        """Rebuild fragment dest[o] of each object into out[o] (header included)."""
        n_obj = len(avail_masks)
        if len(dest) != n_obj:
            _native.raise_error(-_native.EINVALIDPARAMS, "ecamd_reconstruct_batch")
        self._check_count("ecamd_reconstruct_batch", n_obj, frags, out)
        for x in (frags, out):
            self._check_rows("ecamd_reconstruct_batch", x)
        masks = (ctypes.c_uint32 * n_obj)(*avail_masks)
        dst = (ctypes.c_int * n_obj)(*dest)
        fs = int(frags.stride(1))
        ret = _native.lib.ecamd_reconstruct_batch(
            self.handle.desc, _ptr(frags), fs, _stride0(frags, (self.k + self.m) * fs), obj_len,
            n_obj, masks, dst, _ptr(out), _stride0(out, fs), _stream(stream))
        self._check(ret, "ecamd_reconstruct_batch")

    def encode_host(self, objs: Any, obj_len: int, parity: Any) -> None:
        """Host-resident encode: objs (n_obj, obj_stride) and parity
        (n_obj, m, frag_stride) in (pinned) host memory."""
        n_obj = int(objs.shape[0])
        self._check_count("ecamd_encode_host_batch", n_obj, parity)
        self._check_rows("ecamd_encode_host_batch", objs)
        self._check_rows("ecamd_encode_host_batch", parity, self.m)
        ret = _native.lib.ecamd_encode_host_batch(
            self.handle.desc, _ptr(objs), _stride0(objs, obj_len), obj_len, n_obj,
            _ptr(parity), int(parity.stride(1)))
        self._check(ret, "ecamd_encode_host_batch")

    def decode_host(self, frags: Any, obj_len: int, avail_masks: Sequence[int],
                    out: Any) -> None:
        """Host-resident decode.  frags: (n_obj, k, frag_stride) (pinned) host
        tensor holding, per object, the fragments named by the k lowest set
        bits of its mask in ascending index order; out: (n_obj, obj_stride)."""
        n_obj = len(avail_masks)
        self._check_count("ecamd_decode_host_batch", n_obj, frags, out)
        if hasattr(frags, "shape") and int(frags.shape[1]) != self.k:
            _native.raise_error(-_native.EINVALIDPARAMS, "ecamd_decode_host_batch")
        self._check_rows("ecamd_decode_host_batch", frags, self.k)
        self._check_rows("ecamd_decode_host_batch", out)
        masks = (ctypes.c_uint32 * n_obj)(*avail_masks)
        ret = _native.lib.ecamd_decode_host_batch(
            self.handle.desc, _ptr(frags), int(frags.stride(1)), obj_len, n_obj, masks,
            _ptr(out), _stride0(out, obj_len))
        self._check(ret, "ecamd_decode_host_batch")

    def reconstruct_host(self, frags: Any, obj_len: int, avail_masks: Sequence[int],
                         dest: Sequence[int], out: Any) -> None:
        """Host-resident reconstruct: inputs as decode_host; fragment dest[o]
        (header included) into out[o] ((n_obj, frag_stride) host tensor)."""
        n_obj = len(avail_masks)
        if len(dest) != n_obj or (hasattr(frags, "shape") and int(frags.shape[1]) != self.k):
            _native.raise_error(-_native.EINVALIDPARAMS, "ecamd_reconstruct_host_batch")
        self._check_count("ecamd_reconstruct_host_batch", n_obj, frags, out)
        self._check_rows("ecamd_reconstruct_host_batch", frags, self.k)
        self._check_rows("ecamd_reconstruct_host_batch", out)
        masks = (ctypes.c_uint32 * n_obj)(*avail_masks)
        dst = (ctypes.c_int * n_obj)(*dest)
        ret = _native.lib.ecamd_reconstruct_host_batch(
            self.handle.desc, _ptr(frags), int(frags.stride(1)), obj_len, n_obj, masks, dst,
            _ptr(out), _stride0(out, 0))
        self._check(ret, "ecamd_reconstruct_host_batch")
