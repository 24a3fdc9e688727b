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
HEADER = os.path.join(os.path.dirname(HERE), "include", "nvl_crc32c.h")

OK = 0
EINVAL = -1
EHIP = -2
ENODEV = -3
ESELFTEST = -4
ENOSPC = -5
FLAG_MASK = 0x1

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
    "nvl_crc32c_extend": (_u32, [_u32, _vp, _sz]),
    "nvl_crc32c_value": (_u32, [_vp, _sz]),
    "nvl_crc32c_mask": (_u32, [_u32]),
    "nvl_crc32c_unmask": (_u32, [_u32]),
    "nvl_crc32c_fixed_dev": (_int, [_vp, _u64, _u64, _u64, _vp, _u32, _vp, _u32, _vp, _sz, _vp]),
    "nvl_crc32c_fixed_workspace_bytes": (_sz, [_u64, _u64, _u64]),
    "nvl_crc32c_batch_dev": (_int, [_vp, _vp, _vp, _vp, _u32, _vp, _u64, _u32, _vp, _sz, _vp]),
    "nvl_crc32c_batch_workspace_bytes": (_sz, [_u64]),
    "nvl_crc32c_batch_host": (_int, [_vp, _vp, _vp, _u32, _vp, _u64, _u32]),
    "nvl_crc32c_fixed_host": (_int, [_vp, _u64, _u64, _u64, _vp, _u32, _vp, _u32]),
    "nvl_crc32c_fill_splitmix": (_int, [_vp, _u64, _u64, _u64, _u64, _u64, _vp]),
}


def header_symbols(path: str = HEADER) -> list[str]:
    """Every entry point the C header declares (NVL_API ... nvl_crc32c_x(...))."""
    with open(path) as f:
        text = f.read()
    return sorted(set(re.findall(r"NVL_API[^;(]*?\b(nvl_crc32c_\w+)\s*\(", text)))


def load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C nvlevelz_amd/csrc` (the batch CRC32C path has no fallback)")
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
