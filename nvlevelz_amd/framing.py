"""Python view of the call-site shims (include/nvl_framing.h): SSTable block
trailers, block and whole-table verification, log scan and log sealing, each
one CRC batch: by default the library's size policy picks the calling
thread's host CRC or the GPU (nvl_framing_uses_gpu);
``host=True`` forces the host CRC, ``host=False`` the GPU.

Verdicts carry the reference's Status texts, so a caller can report them the
way LevelDB does:

* ReadBlock, table/format.cc:65-98 -- "truncated block read",
  "block checksum mismatch", "bad block type";
* Table::Open, table/table.cc:38-82, and Block::Iter, table/block.cc --
  "file is too short to be an sstable", "not an sstable (bad magic number)",
  "bad block handle", "bad block contents", "bad entry in block";
* log::Reader::ReadPhysicalRecord, db/log_reader.cc:199-281 -- the per-record
  outcomes of nvl_log_scan.

Every function raises :class:`FramingError` on a non-OK return code; there is
no silent fallback (without a GPU the device mode raises).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, List, Sequence, Tuple, Union

import numpy as np

from . import _lib

BytesLike = Union[bytes, bytearray, memoryview, np.ndarray]

BLOCK_TEXT = {
    _lib.BLOCK_OK: "OK",
    _lib.BLOCK_TRUNCATED: "Corruption: truncated block read",
    _lib.BLOCK_CHECKSUM_MISMATCH: "Corruption: block checksum mismatch",
    _lib.BLOCK_BAD_TYPE: "Corruption: bad block type",
    _lib.BLOCK_BAD_HANDLE: "Corruption: bad block handle",
}
TABLE_TEXT = {
    _lib.TABLE_OK: "OK",
    _lib.TABLE_TOO_SHORT: "Corruption: file is too short to be an sstable",
    _lib.TABLE_BAD_MAGIC: "Corruption: not an sstable (bad magic number)",
    _lib.TABLE_BAD_FOOTER: "Corruption: bad block handle",
    _lib.TABLE_INDEX_UNREADABLE: "index block unreadable",  # blocks[0] carries the ReadBlock text
    _lib.TABLE_BAD_INDEX_BLOCK: "Corruption: bad block contents",
    _lib.TABLE_BAD_INDEX_ENTRY: "Corruption: bad entry in block",
    _lib.TABLE_COMPRESSED_INDEX: "index block is compressed (not parsed)",
}
ROLE_TEXT = {_lib.TBLOCK_INDEX: "index", _lib.TBLOCK_METAINDEX: "metaindex", _lib.TBLOCK_META: "meta",
             _lib.TBLOCK_DATA: "data"}


class FramingError(RuntimeError):
    def __init__(self, rc: int, what: str):
        super().__init__(f"{what}: {_lib.lib.nvl_crc32c_strerror(rc).decode()} ({rc})")
        self.rc = rc


def _flags(host) -> int:
    """host=None: the library's size policy (nvl_framing_uses_gpu); True: the
    host CRC; False: the GPU whatever the size."""
    if host is None:
        return 0
    return _lib.FRAMING_HOST if host else _lib.FRAMING_GPU


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise FramingError(rc, what)


def _handles(handles) -> np.ndarray:
    h = np.ascontiguousarray(np.asarray(handles, dtype=np.uint64).reshape(-1, 2))
    return h


def _ro(data: BytesLike):
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        return a.ctypes.data, a.size, a
    if isinstance(data, memoryview):
        data = data.tobytes()
    if isinstance(data, bytearray):
        return (ctypes.c_char * len(data)).from_buffer(data), len(data), data
    return data, len(data), data


def seal_trailers(image: Union[bytearray, np.ndarray], handles, *, host: Optional[bool] = None) -> None:
    """TableBuilder::WriteRawBlock's trailer (table/table_builder.cc:183-188) for
    every (offset, size) handle, in place: image[off+size] holds the type,
    Mask(Value(block | type)) goes to image[off+size+1 .. +5)."""
    h = _handles(handles)
    if isinstance(image, np.ndarray):
        ptr, n = image.ctypes.data, image.nbytes
    elif isinstance(image, bytearray):
        ptr, n = (ctypes.c_char * len(image)).from_buffer(image), len(image)
    else:
        raise TypeError("seal_trailers writes in place: pass a bytearray or a numpy array")
    _check(_lib.lib.nvl_sstable_seal_trailers(ptr, n, h.ctypes.data, len(h), _flags(host)), "seal_trailers")


def verify_blocks(image: BytesLike, handles, *, host: Optional[bool] = None) -> np.ndarray:
    """ReadBlock's checks (verify_checksums) for every handle: an array of
    NVL_BLOCK_* verdicts (see BLOCK_TEXT)."""
    h = _handles(handles)
    ptr, n, _keep = _ro(image)
    v = np.zeros(len(h), dtype=np.uint8)
    bad = ctypes.c_uint64(0)
    _check(_lib.lib.nvl_sstable_verify_blocks(ptr, n, h.ctypes.data, len(h), v.ctypes.data, ctypes.byref(bad),
                                              _flags(host)), "verify_blocks")
    return v


@dataclass
class TableBlockReport:
    offset: int
    size: int
    role: str
    verdict: int

    @property
    def text(self) -> str:
        return BLOCK_TEXT[self.verdict]


@dataclass
class TableReport:
    status: int
    blocks: List[TableBlockReport]

    @property
    def ok(self) -> bool:
        return self.status == _lib.TABLE_OK and all(b.verdict == _lib.BLOCK_OK for b in self.blocks)

    @property
    def status_text(self) -> str:
        if self.status == _lib.TABLE_INDEX_UNREADABLE and self.blocks:
            return self.blocks[0].text
        return TABLE_TEXT[self.status]

    def bad(self) -> List[TableBlockReport]:
        return [b for b in self.blocks if b.verdict != _lib.BLOCK_OK]


def verify_table(image: BytesLike, *, host: Optional[bool] = None) -> TableReport:
    """Every block of an SSTable image verified in one batch
    (nvl_sstable_verify_table): index, metaindex, meta blocks, data blocks."""
    ptr, n, _keep = _ro(image)
    cnt = ctypes.c_size_t(0)
    st = ctypes.c_uint32(0)
    bad = ctypes.c_uint64(0)
    # one call when the guess fits: the index holds at most one handle per 3+2 bytes
    cap = max(16, min(n // 5 + 8, 1 << 22))
    while True:
        arr = (_lib.TableBlock * cap)()
        rc = _lib.lib.nvl_sstable_verify_table(ptr, n, arr, cap, ctypes.byref(cnt), ctypes.byref(st),
                                               ctypes.byref(bad), _flags(host))
        if rc == _lib.ENOSPC and cnt.value > cap:
            cap = cnt.value
            continue
        _check(rc, "verify_table")
        break
    blocks = [TableBlockReport(a.offset, a.size, ROLE_TEXT[a.role], a.verdict) for a in arr[:cnt.value]]
    return TableReport(st.value, blocks)


def verify_table_dev(image, stream=None) -> TableReport:
    """verify_table for an SSTable image already in device memory: a 1-D
    uint8 torch tensor on the GPU (nvl_sstable_verify_table_dev; only the
    footer, index and metaindex come back to the host)."""
    import torch
    if not (isinstance(image, torch.Tensor) and image.is_cuda and image.dtype == torch.uint8 and image.dim() == 1
            and image.is_contiguous()):
        raise TypeError("verify_table_dev: a contiguous 1-D uint8 tensor on the GPU")
    st_ = torch.cuda.current_stream(image.device).cuda_stream if stream is None else stream
    n = image.numel()
    cnt = ctypes.c_size_t(0)
    st = ctypes.c_uint32(0)
    bad = ctypes.c_uint64(0)
    with torch.cuda.device(image.device):
        _check(_lib.lib.nvl_sstable_verify_table_dev(image.data_ptr(), n, None, 0, ctypes.byref(cnt), ctypes.byref(st),
                                                     ctypes.byref(bad), st_), "verify_table_dev")
        cap = max(cnt.value, 1)
        arr = (_lib.TableBlock * cap)()
        _check(_lib.lib.nvl_sstable_verify_table_dev(image.data_ptr(), n, arr, cap, ctypes.byref(cnt), ctypes.byref(st),
                                                     ctypes.byref(bad), st_), "verify_table_dev")
    blocks = [TableBlockReport(a.offset, a.size, ROLE_TEXT[a.role], a.verdict) for a in arr[:cnt.value]]
    return TableReport(st.value, blocks)


LOG_KIND = {_lib.LOG_RECORD: "record", _lib.LOG_BAD_LENGTH: "bad record length",
            _lib.LOG_CHECKSUM: "checksum mismatch", _lib.LOG_ZERO: "zero", _lib.LOG_EOF: "eof"}


def log_scan(image: BytesLike, *, start: int = 0, checksum: bool = True,
             host: Optional[bool] = None) -> List[Tuple[str, int, int, int]]:
    """ReadPhysicalRecord's outcomes over a log image (nvl_log_scan):
    [(kind, header_offset, payload_length, type)] ending with ("eof", ...)."""
    ptr, n, _keep = _ro(image)
    cnt = ctypes.c_size_t(0)
    # One scan when the guess fits (records of >= ~256 B on average); a log of
    # tinier records is scanned again with the exact count the first call reported.
    cap = n // 256 + 64
    while True:
        ev = (_lib.LogEvent * cap)()
        rc = _lib.lib.nvl_log_scan(ptr, n, start, int(checksum), ev, cap, ctypes.byref(cnt), _flags(host))
        if rc == _lib.ENOSPC and cnt.value > cap:
            cap = cnt.value
            continue
        _check(rc, "log_scan")
        break
    return [(LOG_KIND[e.kind], e.offset, e.length, e.type) for e in ev[:cnt.value]]


def log_seal(image: Union[bytearray, np.ndarray], header_offsets: Sequence[int], *, host: Optional[bool] = None) -> None:
    """log::Writer's header CRCs (db/log_writer.cc:93-97) for every header offset, in place."""
    off = np.ascontiguousarray(np.asarray(header_offsets, dtype=np.uint64))
    if isinstance(image, np.ndarray):
        ptr, n = image.ctypes.data, image.nbytes
    elif isinstance(image, bytearray):
        ptr, n = (ctypes.c_char * len(image)).from_buffer(image), len(image)
    else:
        raise TypeError("log_seal writes in place: pass a bytearray or a numpy array")
    _check(_lib.lib.nvl_log_seal(ptr, n, off.ctypes.data, len(off), _flags(host)), "log_seal")
