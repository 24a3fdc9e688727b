"""nvlevelz_amd.crc32c -- Python mirror of the reference's util/crc32c.h API
plus the batched device-resident engine behind it.

Reference interface (/root/reference/util/crc32c.h):
    Extend(init_crc, data, n)  -> :func:`extend`       (crc32c.h:17)
    Value(data, n)             -> :func:`value`        (crc32c.h:20-22)
    kMaskDelta                 -> :data:`kMaskDelta`   (crc32c.h:24)
    Mask(crc) / Unmask(m)      -> :func:`mask` / :func:`unmask` (crc32c.h:31-40)

Batched, MI355X-resident (the hot path; HIP kernels via the C ABI):
    :func:`extend_fixed`  -- n buffers at a fixed stride (SSTable data blocks,
                             db_bench's 4 KiB crc32c loop)
    :func:`extend_batch`  -- n buffers at arbitrary offsets/lengths
    :func:`extend_batch_host`, :func:`extend_fixed_host` -- host memory in/out
                             (pinned staging + H2D + kernel + D2H)

The batch functions never fall back to the CPU: without a GPU, or if the
GPU backend fails its known-answer probe (util/crc32c.cc:290-297 analogue),
they raise :class:`Crc32cError`.
"""
from __future__ import annotations

from typing import Optional, Sequence, Union

import numpy as np

from . import _lib
from ._lib import Crc32cError, FLAG_MASK, check, lib

kMaskDelta = 0xA282EAD8

BytesLike = Union[bytes, bytearray, memoryview, np.ndarray]


def _buf(data: BytesLike):
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8)
        return a, a.ctypes.data, a.nbytes
    b = bytes(data)
    return b, b, len(b)


# ---- util/crc32c.h API (host, one buffer) ---------------------------------

def extend(init_crc: int, data: BytesLike) -> int:
    """crc32c of concat(A, data) given init_crc = crc32c(A) (util/crc32c.h:14-17)."""
    keep, ptr, n = _buf(data)
    return lib.nvl_crc32c_extend(init_crc & 0xFFFFFFFF, ptr, n)


def value(data: BytesLike) -> int:
    """crc32c of data (util/crc32c.h:20-22)."""
    keep, ptr, n = _buf(data)
    return lib.nvl_crc32c_value(ptr, n)


def mask(crc: int) -> int:
    """Masked representation of crc: rotate right 15, add kMaskDelta (util/crc32c.h:31-34)."""
    return lib.nvl_crc32c_mask(crc & 0xFFFFFFFF)


def unmask(masked_crc: int) -> int:
    """Inverse of :func:`mask` (util/crc32c.h:37-40)."""
    return lib.nvl_crc32c_unmask(masked_crc & 0xFFFFFFFF)


# ---- device-resident batches ----------------------------------------------

def _torch():
    import torch  # plumbing only: device memory + streams
    return torch


def init(device: int = 0) -> None:
    """Build tables on `device` and run the GPU known-answer probe."""
    check(lib.nvl_crc32c_init(device), "nvl_crc32c_init")


def gpu_accelerated() -> bool:
    return bool(lib.nvl_crc32c_gpu_accelerated())


def _stream_handle(t) -> int:
    torch = _torch()
    return torch.cuda.current_stream(t.device).cuda_stream


def _require_dev(t, name: str, dtype=None, device=None):
    """A contiguous HIP tensor of an allowed dtype, on `device` when given
    (every operand of a batch lives on the device of the launch stream)."""
    torch = _torch()
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA(HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype not in dtype:
        raise TypeError(f"{name} has dtype {t.dtype}, expected one of {dtype}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, the batch on {device}")


def fixed_workspace_bytes(stride: int, length: int, n: int) -> int:
    return lib.nvl_crc32c_fixed_workspace_bytes(stride, length, n)


def batch_workspace_bytes(n: int) -> int:
    return lib.nvl_crc32c_batch_workspace_bytes(n)


def extend_fixed(buf, stride: int, length: int, n: int, init=0, *, mask: bool = False,
                 base_offset: int = 0, out=None, workspace=None):
    """out[i] = Extend(init_i, buf[base_offset + i*stride : ... + length]).

    ``buf`` is a uint8 device tensor; ``init`` an int (all buffers) or an
    int32/uint32 device tensor of n values.  Returns an int32 device tensor
    holding the u32 results (bit pattern).  Asynchronous on the current stream.
    """
    torch = _torch()
    _require_dev(buf, "buf", (torch.uint8, torch.int8))
    if n < 0 or length < 0 or stride < 0 or base_offset < 0:
        raise ValueError("negative size")
    if n and base_offset + (n - 1) * stride + length > buf.numel():
        raise ValueError("batch extends past the end of buf")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=buf.device)
    _require_dev(out, "out", (torch.int32, torch.uint32), buf.device)
    if out.numel() < n:
        raise ValueError("out too small")
    init_ptr, init_all = None, 0
    if isinstance(init, int):
        init_all = init & 0xFFFFFFFF
    else:
        _require_dev(init, "init", (torch.int32, torch.uint32), buf.device)
        if init.numel() < n:
            raise ValueError("init too small")
        init_ptr = init.data_ptr()
    ws_ptr, ws_bytes = None, 0
    if workspace is not None:
        ws_ptr, ws_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    rc = lib.nvl_crc32c_fixed_dev(buf.data_ptr() + base_offset, stride, length, n, init_ptr, init_all,
                                  out.data_ptr(), FLAG_MASK if mask else 0, ws_ptr, ws_bytes,
                                  _stream_handle(buf))
    check(rc, "nvl_crc32c_fixed_dev")
    return out


class FixedBatch:
    """A validated fixed-stride batch whose launch does no host work beyond the
    C call: arguments are checked and converted once, the workspace is sized
    once, and :meth:`launch` re-enqueues the same batch on the same stream
    (e.g. a table's blocks re-verified, or the bench loop).  The output is
    ``self.out`` (int32 device tensor holding the u32 bit patterns)."""

    def __init__(self, buf, stride: int, length: int, n: int, init=0, *, mask: bool = False,
                 base_offset: int = 0, out=None, workspace=None, stream=None):
        torch = _torch()
        _require_dev(buf, "buf", (torch.uint8, torch.int8))
        if n < 0 or length < 0 or stride < 0 or base_offset < 0:
            raise ValueError("negative size")
        if n and base_offset + (n - 1) * stride + length > buf.numel():
            raise ValueError("batch extends past the end of buf")
        self.buf = buf
        self.out = out if out is not None else torch.empty(n, dtype=torch.int32, device=buf.device)
        _require_dev(self.out, "out", (torch.int32, torch.uint32), buf.device)
        if self.out.numel() < n:
            raise ValueError("out too small")
        self.init = init
        init_ptr, init_all = None, 0
        if isinstance(init, int):
            init_all = init & 0xFFFFFFFF
        else:
            _require_dev(init, "init", (torch.int32, torch.uint32), buf.device)
            if init.numel() < n:
                raise ValueError("init too small")
            init_ptr = init.data_ptr()
        need = lib.nvl_crc32c_fixed_workspace_bytes(stride, length, n)
        if workspace is None and need:
            workspace = torch.empty(need, dtype=torch.uint8, device=buf.device)
        self.workspace = workspace
        ws_ptr, ws_bytes = None, 0
        if workspace is not None:
            ws_ptr, ws_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
        if stream is None:
            stream = torch.cuda.current_stream(buf.device)
        if stream.device != buf.device:
            raise ValueError(f"stream is on {stream.device}, buf on {buf.device}")
        self.stream = stream
        self._args = (buf.data_ptr() + base_offset, stride, length, n, init_ptr, init_all,
                      self.out.data_ptr(), FLAG_MASK if mask else 0, ws_ptr, ws_bytes, stream.cuda_stream)
        self._fn = lib.nvl_crc32c_fixed_dev

    def launch(self):
        rc = self._fn(*self._args)
        if rc:
            check(rc, "nvl_crc32c_fixed_dev")
        return self.out

    def launch_timed(self, start, stop):
        """:meth:`launch` through nvl_crc32c_fixed_dev_timed: the kernel
        dispatch itself records ``start``/``stop`` (torch.cuda.Event with
        timing, already materialised by one ``record()``), so their elapsed
        time is the kernel's own duration and nothing is enqueued between
        back-to-back launches."""
        rc = lib.nvl_crc32c_fixed_dev_timed(*self._args, start.cuda_event, stop.cuda_event)
        if rc:
            check(rc, "nvl_crc32c_fixed_dev_timed")
        return self.out


def extend_batch(buf, offsets, lengths, init=0, *, mask: bool = False, out=None, workspace=None):
    """out[i] = Extend(init_i, buf[offsets[i] : offsets[i] + lengths[i]]).

    ``offsets``/``lengths`` are int64 device tensors (u64 bit patterns).
    Arbitrary alignment and lengths (0 included).  Asynchronous.
    """
    torch = _torch()
    _require_dev(buf, "buf", (torch.uint8, torch.int8))
    _require_dev(offsets, "offsets", (torch.int64, torch.uint64), buf.device)
    _require_dev(lengths, "lengths", (torch.int64, torch.uint64), buf.device)
    n = offsets.numel()
    if lengths.numel() != n:
        raise ValueError("offsets and lengths differ in size")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=buf.device)
    _require_dev(out, "out", (torch.int32, torch.uint32), buf.device)
    if out.numel() < n:
        raise ValueError("out too small")  # the kernel writes n results
    init_ptr, init_all = None, 0
    if isinstance(init, int):
        init_all = init & 0xFFFFFFFF
    else:
        _require_dev(init, "init", (torch.int32, torch.uint32), buf.device)
        if init.numel() < n:
            raise ValueError("init too small")  # the kernel reads n values
        init_ptr = init.data_ptr()
    ws_ptr, ws_bytes = None, 0
    if workspace is not None:
        _require_dev(workspace, "workspace", None, buf.device)
        ws_ptr, ws_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    rc = lib.nvl_crc32c_batch_dev(buf.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), init_ptr, init_all,
                                  out.data_ptr(), n, FLAG_MASK if mask else 0, ws_ptr, ws_bytes,
                                  _stream_handle(buf))
    check(rc, "nvl_crc32c_batch_dev")
    return out


def region_workspace_bytes(region_len: int, n: int) -> int:
    return int(lib.nvl_crc32c_region_workspace_bytes(region_len, n))


def extend_region(buf, offsets, lengths, init=0, *, mask: bool = False, out=None, workspace=None,
                  shaped: bool = False):
    """out[i] = Extend(init_i, buf[offsets[i] : offsets[i] + lengths[i]]) for
    buffers inside ``buf`` sorted by offset and non-overlapping (an SSTable
    image's blocks, a packed batch): nvl_crc32c_region_dev, which reads the
    whole of ``buf`` in page-aligned 4 KiB chunks.  The layout is checked on
    the device (other layouts run the batch kernels); ``shaped=True``
    (NVL_CRC32C_FLAG_REGION_SHAPED) skips the check for a caller that has made
    it itself -- one launch, and a slow per-buffer path if it was wrong.
    Asynchronous."""
    torch = _torch()
    _require_dev(buf, "buf", (torch.uint8, torch.int8))
    _require_dev(offsets, "offsets", (torch.int64, torch.uint64), buf.device)
    _require_dev(lengths, "lengths", (torch.int64, torch.uint64), buf.device)
    n = offsets.numel()
    if lengths.numel() != n:
        raise ValueError("offsets and lengths differ in size")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=buf.device)
    _require_dev(out, "out", (torch.int32, torch.uint32), buf.device)
    if out.numel() < n:
        raise ValueError("out too small")
    init_ptr, init_all = None, 0
    if isinstance(init, int):
        init_all = init & 0xFFFFFFFF
    else:
        _require_dev(init, "init", (torch.int32, torch.uint32), buf.device)
        if init.numel() < n:
            raise ValueError("init too small")
        init_ptr = init.data_ptr()
    ws_ptr, ws_bytes = None, 0
    if workspace is not None:
        _require_dev(workspace, "workspace", None, buf.device)
        ws_ptr, ws_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    flags = (FLAG_MASK if mask else 0) | (_lib.FLAG_REGION_SHAPED if shaped else 0)
    rc = lib.nvl_crc32c_region_dev(buf.data_ptr(), buf.numel(), offsets.data_ptr(), lengths.data_ptr(), init_ptr,
                                   init_all, out.data_ptr(), n, flags, ws_ptr, ws_bytes, _stream_handle(buf))
    check(rc, "nvl_crc32c_region_dev")
    return out


def extend_batch_host(buffers: Sequence[BytesLike], init: Union[int, Sequence[int]] = 0, *,
                      mask: bool = False) -> np.ndarray:
    """Host buffers in, u32 CRCs out (synchronous; pinned staging + GPU)."""
    import ctypes
    n = len(buffers)
    keep = [_buf(b) for b in buffers]
    ptrs = (ctypes.c_void_p * max(n, 1))()
    lens = np.empty(n, dtype=np.uint64)
    for i, (obj, p, m) in enumerate(keep):
        ptrs[i] = ctypes.cast(ctypes.c_char_p(obj), ctypes.c_void_p).value if isinstance(obj, bytes) else p
        lens[i] = m
    out = np.empty(n, dtype=np.uint32)
    init_ptr, init_all = None, 0
    if isinstance(init, int):
        init_all = init & 0xFFFFFFFF
    else:
        ini = np.ascontiguousarray(np.asarray(init, dtype=np.uint64) & 0xFFFFFFFF, dtype=np.uint32)
        init_ptr = ini.ctypes.data
    rc = lib.nvl_crc32c_batch_host(ptrs, lens.ctypes.data, init_ptr, init_all, out.ctypes.data, n,
                                   FLAG_MASK if mask else 0)
    check(rc, "nvl_crc32c_batch_host")
    return out


def extend_fixed_host(buf: np.ndarray, stride: int, length: int, n: int, init=0, *,
                      mask: bool = False) -> np.ndarray:
    """Fixed-stride batch over one contiguous host region (pinned is fastest)."""
    a = buf if isinstance(buf, np.ndarray) else np.frombuffer(buf, dtype=np.uint8)
    if n and (n - 1) * stride + length > a.nbytes:
        raise ValueError("batch extends past the end of buf")
    out = np.empty(n, dtype=np.uint32)
    init_ptr, init_all = None, 0
    if isinstance(init, int):
        init_all = init & 0xFFFFFFFF
    else:
        ini = np.ascontiguousarray(np.asarray(init, dtype=np.uint64) & 0xFFFFFFFF, dtype=np.uint32)
        init_ptr = ini.ctypes.data
    rc = lib.nvl_crc32c_fixed_host(a.ctypes.data, stride, length, n, init_ptr, init_all, out.ctypes.data,
                                   FLAG_MASK if mask else 0)
    check(rc, "nvl_crc32c_fixed_host")
    return out


def host_register(arr) -> None:
    """nvl_crc32c_host_register over a host array's bytes (numpy array or
    buffer): pinned and mapped for every device until host_unregister, so
    extend_region_host DMAs straight from it (no staging copy) or, with
    ``zero_copy=True``, reads it in place.  The caller keeps ``arr`` alive."""
    a = arr if isinstance(arr, np.ndarray) else np.frombuffer(arr, dtype=np.uint8)
    check(lib.nvl_crc32c_host_register(a.ctypes.data, a.nbytes), "nvl_crc32c_host_register")


def host_unregister(arr) -> None:
    a = arr if isinstance(arr, np.ndarray) else np.frombuffer(arr, dtype=np.uint8)
    check(lib.nvl_crc32c_host_unregister(a.ctypes.data), "nvl_crc32c_host_unregister")


def host_registered(arr) -> bool:
    a = arr if isinstance(arr, np.ndarray) else np.frombuffer(arr, dtype=np.uint8)
    return lib.nvl_crc32c_host_registered(a.ctypes.data, a.nbytes) == 1


def extend_region_host(region: np.ndarray, offsets, lengths, init=0, *, mask: bool = False,
                       devices: Optional[Sequence[int]] = None, min_bytes_per_device: int = 0,
                       zero_copy: bool = False) -> np.ndarray:
    """out[i] = Extend(init_i, region[offsets[i] : offsets[i] + lengths[i]]) for
    buffers in ONE host region (an mmap'd file image, a log block run):
    nvl_crc32c_batch_region_host on the current device, or with ``devices``
    nvl_crc32c_batch_region_host_multi -- contiguous ranges of the batch on
    those devices at once, each over its own PCIe link (synchronous).  A
    region inside a host_register()ed range is DMA'd from its own pages (no
    staging copy); ``zero_copy`` (registered ranges only) has the kernels read
    it in place over PCIe."""
    a = region if isinstance(region, np.ndarray) else np.frombuffer(region, dtype=np.uint8)
    a = np.ascontiguousarray(a).view(np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    m = np.ascontiguousarray(lengths, dtype=np.uint64)
    n = o.size
    if m.size != n:
        raise ValueError("offsets and lengths differ in size")
    out = np.empty(n, dtype=np.uint32)
    init_ptr, init_all = None, 0
    if isinstance(init, int):
        init_all = init & 0xFFFFFFFF
    else:
        ini = np.ascontiguousarray(np.asarray(init, dtype=np.uint64) & 0xFFFFFFFF, dtype=np.uint32)
        init_ptr = ini.ctypes.data
    flags = (FLAG_MASK if mask else 0) | (_lib.FLAG_HOST_ZERO_COPY if zero_copy else 0)
    if devices is None:
        rc = lib.nvl_crc32c_batch_region_host(a.ctypes.data, a.nbytes, o.ctypes.data, m.ctypes.data, init_ptr,
                                              init_all, out.ctypes.data, n, flags)
        check(rc, "nvl_crc32c_batch_region_host")
    else:
        dv = np.ascontiguousarray(devices, dtype=np.int32)
        rc = lib.nvl_crc32c_batch_region_host_multi(a.ctypes.data, a.nbytes, o.ctypes.data, m.ctypes.data, init_ptr,
                                                    init_all, out.ctypes.data, n, flags, dv.ctypes.data, dv.size,
                                                    min_bytes_per_device)
        check(rc, "nvl_crc32c_batch_region_host_multi")
    return out


def extend_fixed_multi(shards, init: int = 0, *, mask: bool = False):
    """nvl_crc32c_fixed_dev_multi: one fixed-stride batch per device tensor,
    every shard checksummed on the device holding it (one process, no bytes
    cross devices).  shards: [(buf, stride, length, n)], buf a uint8 device
    tensor (its device and current stream are the shard's).  Returns one
    int32 result tensor per shard, on its device; asynchronous like
    extend_fixed (synchronise the shards' streams before reading)."""
    torch = _torch()
    arr = (_lib.Shard * max(len(shards), 1))()
    outs = []
    for k, (buf, stride, length, n) in enumerate(shards):
        _require_dev(buf, "buf", (torch.uint8, torch.int8))
        if n and (n - 1) * stride + length > buf.numel():
            raise ValueError(f"shard {k} extends past the end of its buffer")
        out = torch.empty(max(n, 1), dtype=torch.int32, device=buf.device)[:n]
        outs.append(out)
        arr[k] = _lib.Shard(buf.device.index, buf.data_ptr(), stride, length, n, out.data_ptr(), _stream_handle(buf))
    rc = lib.nvl_crc32c_fixed_dev_multi(arr, len(shards), init & 0xFFFFFFFF, FLAG_MASK if mask else 0)
    check(rc, "nvl_crc32c_fixed_dev_multi")
    return outs


def gather_dev(outs, device: int, *, round_robin: bool = False):
    """nvl_crc32c_gather_dev: the shards' result tensors (extend_fixed_multi's)
    gathered into one int32 tensor on `device` -- concatenated, or with
    round_robin=True in config 5's global order (block i from shard i mod G).
    Peer copies of 4 bytes per block; ordered after each shard's stream."""
    torch = _torch()
    arr = (_lib.Shard * max(len(outs), 1))()
    N = 0
    for k, o in enumerate(outs):
        arr[k] = _lib.Shard(o.device.index, None, 0, 0, o.numel(), o.data_ptr(), _stream_handle(o))
        N += o.numel()
    dst = torch.empty(max(N, 1), dtype=torch.int32, device=torch.device("cuda", device))[:N]
    rc = lib.nvl_crc32c_gather_dev(dst.data_ptr(), device, arr, len(outs),
                                   _lib.GATHER_ROUND_ROBIN if round_robin else _lib.GATHER_CONCAT,
                                   _stream_handle(dst))
    check(rc, "nvl_crc32c_gather_dev")
    return dst


def multi_plan(offsets, lengths, ndev: int, min_bytes: int = 0) -> np.ndarray:
    """nvl_crc32c_multi_plan: the first buffer of each part (+ n at the end)."""
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    m = np.ascontiguousarray(lengths, dtype=np.uint64)
    first = np.zeros(ndev + 1, dtype=np.uint64)
    k = lib.nvl_crc32c_multi_plan(o.ctypes.data, m.ctypes.data, o.size, ndev, min_bytes, first.ctypes.data)
    check(k if k < 0 else 0, "nvl_crc32c_multi_plan")
    return first[:k + 1]


def fill_splitmix(buf, nblocks: int, block_bytes: int, seed: int, *, first_block: int = 0,
                  block_step: int = 1) -> None:
    """Write the canonical synthetic stream into a device tensor:
    block k <- stream bytes [(first_block + k*block_step)*block_bytes, +block_bytes)."""
    torch = _torch()
    _require_dev(buf, "buf", (torch.uint8, torch.int8))
    if nblocks * block_bytes > buf.numel():
        raise ValueError("buf too small")
    rc = lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), nblocks, block_bytes, first_block, block_step,
                                      seed & 0xFFFFFFFFFFFFFFFF, _stream_handle(buf))
    check(rc, "nvl_crc32c_fill_splitmix")


def to_u32(t) -> np.ndarray:
    """Device int32 result tensor -> host np.uint32 array."""
    return t.detach().cpu().numpy().view(np.uint32)


__all__ = ["extend", "value", "mask", "unmask", "kMaskDelta", "init", "gpu_accelerated",
           "extend_fixed", "FixedBatch", "extend_batch", "extend_region", "extend_batch_host", "extend_fixed_host",
           "extend_region_host", "host_register", "host_unregister", "host_registered", "extend_fixed_multi", "gather_dev", "multi_plan", "fixed_workspace_bytes", "batch_workspace_bytes", "fill_splitmix",
           "to_u32", "Crc32cError"]
