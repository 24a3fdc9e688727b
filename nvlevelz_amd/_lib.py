"""ctypes binding of libnvl_crc32c.so (the C ABI in include/nvl_crc32c.h).

This is the same binding a ctypes user of the reference would add
(INTEGRATION.md shows the cgo/JNI/C++ forms).  The library is built in-tree
by ``__graft_entry__.build()`` / ``make -C nvlevelz_amd/csrc``; importing this
module without it raises immediately -- there is no Python or CPU stand-in
for the batch path.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnvl_crc32c.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HEADER = os.path.join(INCLUDE, "nvl_crc32c.h")
HEADERS = [HEADER, os.path.join(INCLUDE, "nvl_framing.h")]

OK = 0
EINVAL = -1
EHIP = -2
ENODEV = -3
ESELFTEST = -4
ENOSPC = -5
FLAG_MASK = 0x1
FLAG_REGION_SHAPED = 0x2  # nvl_crc32c_region_dev: the caller checked the layout (one launch)
FLAG_HOST_ZERO_COPY = 0x4  # host region entry: kernels read the registered pages in place
REGION_MAX_LEN = 128 << 10

_c = ctypes
_vp = _c.c_void_p
_u32 = _c.c_uint32
_u64 = _c.c_uint64
_sz = _c.c_size_t
_int = _c.c_int

# name -> (restype, argtypes); must match include/nvl_crc32c.h
SIGNATURES = {
    "nvl_crc32c_init": (_int, [_int]),
    "nvl_crc32c_shutdown": (_int, []),
    "nvl_crc32c_gpu_accelerated": (_int, []),
    "nvl_crc32c_strerror": (_c.c_char_p, [_int]),
    "nvl_crc32c_abi_version": (_int, []),
    "nvl_crc32c_host_impl": (_c.c_char_p, []),
    "nvl_crc32c_extend": (_u32, [_u32, _vp, _sz]),
    "nvl_crc32c_value": (_u32, [_vp, _sz]),
    "nvl_crc32c_mask": (_u32, [_u32]),
    "nvl_crc32c_unmask": (_u32, [_u32]),
    "nvl_crc32c_fixed_dev": (_int, [_vp, _u64, _u64, _u64, _vp, _u32, _vp, _u32, _vp, _sz, _vp]),
    "nvl_crc32c_fixed_dev_timed": (_int, [_vp, _u64, _u64, _u64, _vp, _u32, _vp, _u32, _vp, _sz, _vp, _vp, _vp]),
    "nvl_crc32c_fixed_workspace_bytes": (_sz, [_u64, _u64, _u64]),
    "nvl_crc32c_batch_dev": (_int, [_vp, _vp, _vp, _vp, _u32, _vp, _u64, _u32, _vp, _sz, _vp]),
    "nvl_crc32c_batch_workspace_bytes": (_sz, [_u64]),
    "nvl_crc32c_batch_host": (_int, [_vp, _vp, _vp, _u32, _vp, _u64, _u32]),
    "nvl_crc32c_fixed_host": (_int, [_vp, _u64, _u64, _u64, _vp, _u32, _vp, _u32]),
    "nvl_crc32c_fill_splitmix": (_int, [_vp, _u64, _u64, _u64, _u64, _u64, _vp]),
    "nvl_crc32c_read_probe": (_int, [_vp, _u64, _vp, _vp]),
    "nvl_crc32c_batch_region_host": (_int, [_vp, _u64, _vp, _vp, _vp, _u32, _vp, _u64, _u32]),
    "nvl_crc32c_batch_region_host_multi": (_int, [_vp, _u64, _vp, _vp, _vp, _u32, _vp, _u64, _u32, _vp, _int, _u64]),
    "nvl_crc32c_multi_plan": (_int, [_vp, _vp, _u64, _int, _u64, _vp]),
    "nvl_crc32c_region_dev": (_int, [_vp, _u64, _vp, _vp, _vp, _u32, _vp, _u64, _u32, _vp, _sz, _vp]),
    "nvl_crc32c_region_dev_timed": (_int, [_vp, _u64, _vp, _vp, _vp, _u32, _vp, _u64, _u32, _vp, _sz, _vp, _vp,
                                           _vp]),
    "nvl_crc32c_region_workspace_bytes": (_sz, [_u64, _u64]),
    "nvl_crc32c_host_register": (_int, [_vp, _sz]),
    "nvl_crc32c_fixed_dev_multi": (_int, [_vp, _int, _u32, _u32]),
    "nvl_crc32c_gather_dev": (_int, [_vp, _int, _vp, _int, _u32, _vp]),
    "nvl_crc32c_host_unregister": (_int, [_vp]),
    "nvl_crc32c_host_registered": (_int, [_vp, _sz]),
    # include/nvl_framing.h
    "nvl_framing_gpu_min_bytes": (_u64, []),
    "nvl_framing_uses_gpu": (_int, [_u64, _u32]),
    "nvl_sstable_seal_trailers": (_int, [_vp, _u64, _vp, _sz, _u32]),
    "nvl_sstable_verify_blocks": (_int, [_vp, _u64, _vp, _sz, _vp, _vp, _u32]),
    "nvl_log_scan": (_int, [_vp, _u64, _u64, _int, _vp, _sz, _vp, _u32]),
    "nvl_log_seal": (_int, [_vp, _u64, _vp, _sz, _u32]),
    "nvl_sstable_verify_table": (_int, [_vp, _u64, _vp, _sz, _vp, _vp, _vp, _u32]),
    "nvl_sstable_verify_table_dev": (_int, [_vp, _u64, _vp, _sz, _vp, _vp, _vp, _vp]),
}

FRAMING_HOST = 0x100
FRAMING_GPU = 0x400
BLOCK_OK, BLOCK_TRUNCATED, BLOCK_CHECKSUM_MISMATCH, BLOCK_BAD_TYPE = 0, 1, 2, 3
LOG_RECORD, LOG_BAD_LENGTH, LOG_CHECKSUM, LOG_ZERO, LOG_EOF = 0, 1, 2, 3, 4
BLOCK_BAD_HANDLE = 4
(TABLE_OK, TABLE_TOO_SHORT, TABLE_BAD_MAGIC, TABLE_BAD_FOOTER, TABLE_INDEX_UNREADABLE, TABLE_BAD_INDEX_BLOCK,
 TABLE_BAD_INDEX_ENTRY, TABLE_COMPRESSED_INDEX) = range(8)
TBLOCK_INDEX, TBLOCK_METAINDEX, TBLOCK_META, TBLOCK_DATA = 0, 1, 2, 3


GATHER_CONCAT, GATHER_ROUND_ROBIN = 0, 1


class Shard(ctypes.Structure):
    """nvl_crc32c_shard (include/nvl_crc32c.h)."""
    _fields_ = [("device", _int), ("base", _vp), ("stride", _u64), ("len", _u64), ("n", _u64), ("out", _vp),
                ("stream", _vp)]


class TableBlock(ctypes.Structure):
    """nvl_table_block (include/nvl_framing.h)."""
    _fields_ = [("offset", _u64), ("size", _u64), ("role", _u32), ("verdict", _u32)]


class LogEvent(ctypes.Structure):
    """nvl_log_event (include/nvl_framing.h)."""
    _fields_ = [("offset", _u64), ("block_end", _u64), ("length", _u32), ("type", _u32),
                ("kind", _u32), ("reserved", _u32)]


def header_symbols(paths: list[str] | None = None) -> list[str]:
    """Every entry point the C headers declare (NVL_API ... nvl_x(...))."""
    names: set[str] = set()
    for path in paths or HEADERS:
        with open(path) as f:
            names |= set(re.findall(r"NVL_API[^;(]*?\b(nvl_\w+)\s*\(", f.read()))
    return sorted(names)


def load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C nvlevelz_amd/csrc` (the batch CRC32C path has no fallback)")
    # One HIP runtime per process.  PyTorch ships its own libamdhip64; loaded
    # after ours (/opt/rocm's, by path) it becomes a second runtime and the
    # first HIP call here found no device (ENODEV, tools/shim_latency.py).
    # Importing torch first makes our library bind to the copy already loaded.
    try:
        import torch  # noqa: F401
    except Exception:  # noqa: BLE001 -- a C-ABI-only user without torch: /opt/rocm's runtime
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = load()


class Crc32cError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        msg = lib.nvl_crc32c_strerror(status).decode()
        super().__init__(f"{what}: {msg} (status {status})" if what else f"{msg} (status {status})")
        self.status = status


def check(status: int, what: str = "") -> None:
    if status != OK:
        raise Crc32cError(status, what)
