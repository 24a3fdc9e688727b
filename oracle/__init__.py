"""oracle -- CPU checker for the CRC32C hot path.

TEST INFRASTRUCTURE ONLY.  Imported solely by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg.  The
product package ``nvlevelz_amd`` never imports it.

Two checkers are exposed:

* :data:`port` -- ``liboracle.so``, the clean-room C restatement of
  ``util/crc32c.cc:299-347`` (table path) and ``port/port_posix_sse.cc:69-126``
  (SSE4.2 path), see ``oracle/crc32c_oracle.c``.
* :func:`ref` -- ``oracle/_ref/libref_crc32c_{sse,table}.so``: the reference's
  own sources compiled from ``/root/reference`` (``oracle/Makefile``).  Present
  in this container and shipped prebuilt to the GPU box; absent only if never
  built.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build() -> None:
    """Compile liboracle.so (and _ref/ when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


class _Port:
    """ctypes view of liboracle.so (the C restatement)."""

    def __init__(self) -> None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        lib = ctypes.CDLL(path)
        for name in ("oracle_crc32c_extend", "oracle_crc32c_extend_table",
                     "oracle_crc32c_extend_sse"):
            f = getattr(lib, name)
            f.restype = ctypes.c_uint32
            f.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_crc32c_value.restype = ctypes.c_uint32
        lib.oracle_crc32c_value.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_crc32c_mask.restype = ctypes.c_uint32
        lib.oracle_crc32c_mask.argtypes = [ctypes.c_uint32]
        lib.oracle_crc32c_unmask.restype = ctypes.c_uint32
        lib.oracle_crc32c_unmask.argtypes = [ctypes.c_uint32]
        lib.oracle_can_accelerate.restype = ctypes.c_int
        lib.oracle_fill_splitmix.restype = None
        lib.oracle_fill_splitmix.argtypes = [ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_cfg3_lengths.restype = ctypes.c_uint64
        lib.oracle_cfg3_lengths.argtypes = [ctypes.c_uint64, ctypes.c_uint64,
                                            _u64p, ctypes.c_uint64]
        lib.oracle_crc32c_fixed.restype = None
        lib.oracle_crc32c_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_void_p, ctypes.c_void_p]
        lib.oracle_crc32c_varlen.restype = None
        lib.oracle_crc32c_varlen.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_void_p]
        lib.oracle_digest.restype = ctypes.c_uint32
        lib.oracle_digest.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        lib.oracle_crc32c_fixed_mt.restype = ctypes.c_int
        lib.oracle_crc32c_fixed_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_uint64, ctypes.c_uint64,
                                               ctypes.c_void_p, ctypes.c_int,
                                               ctypes.c_int]
        lib.oracle_crc32c_fixed_mt_reps.restype = ctypes.c_int
        lib.oracle_crc32c_fixed_mt_reps.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                                    ctypes.c_uint64, ctypes.c_uint64,
                                                    ctypes.c_void_p, ctypes.c_int,
                                                    ctypes.c_int, ctypes.c_uint64]
        self.lib = lib

    # -- util/crc32c.h API -------------------------------------------------
    def extend(self, init: int, data) -> int:
        b = bytes(data)
        return self.lib.oracle_crc32c_extend(init & 0xFFFFFFFF, b, len(b))

    def extend_table(self, init: int, data) -> int:
        b = bytes(data)
        return self.lib.oracle_crc32c_extend_table(init & 0xFFFFFFFF, b, len(b))

    def extend_sse(self, init: int, data) -> int:
        b = bytes(data)
        return self.lib.oracle_crc32c_extend_sse(init & 0xFFFFFFFF, b, len(b))

    def value(self, data) -> int:
        return self.extend(0, data)

    def mask(self, crc: int) -> int:
        return self.lib.oracle_crc32c_mask(crc & 0xFFFFFFFF)

    def unmask(self, m: int) -> int:
        return self.lib.oracle_crc32c_unmask(m & 0xFFFFFFFF)

    # -- synthetic inputs ------------------------------------
    def fill(self, seed: int, offset: int, n: int) -> np.ndarray:
        out = np.empty(n, dtype=np.uint8)
        self.lib.oracle_fill_splitmix(seed, offset, out.ctypes.data, n)
        return out

    def cfg3_lengths(self, seed: int, total: int) -> np.ndarray:
        k = self.lib.oracle_cfg3_lengths(seed, total, None, 0)
        lens = np.empty(k, dtype=np.uint64)
        self.lib.oracle_cfg3_lengths(seed, total, _ptr(lens, _u64p), k)
        return lens

    # -- batches -------------------------------------------------------------
    def fixed(self, buf: np.ndarray, stride: int, length: int, n: int,
              init: np.ndarray | None = None) -> np.ndarray:
        assert buf.dtype == np.uint8 and buf.flags.c_contiguous
        if n:
            assert (n - 1) * stride + length <= buf.size
        out = np.empty(n, dtype=np.uint32)
        ini = None
        if init is not None:
            init = np.ascontiguousarray(init, dtype=np.uint32)
            ini = init.ctypes.data
        self.lib.oracle_crc32c_fixed(buf.ctypes.data, stride, length, n, ini,
                                     out.ctypes.data)
        return out

    def varlen(self, buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
               init: np.ndarray | None = None) -> np.ndarray:
        assert buf.dtype == np.uint8 and buf.flags.c_contiguous
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        n = offsets.size
        if n:
            assert int((offsets + lengths).max()) <= buf.size
        out = np.empty(n, dtype=np.uint32)
        ini = None
        if init is not None:
            init = np.ascontiguousarray(init, dtype=np.uint32)
            ini = init.ctypes.data
        self.lib.oracle_crc32c_varlen(buf.ctypes.data, offsets.ctypes.data,
                                      lengths.ctypes.data, n, ini, out.ctypes.data)
        return out

    def digest(self, crcs: np.ndarray) -> int:
        crcs = np.ascontiguousarray(crcs, dtype=np.uint32)
        return self.lib.oracle_digest(crcs.ctypes.data, crcs.size)

    def fixed_mt(self, buf: np.ndarray, stride: int, length: int, n: int,
                 threads: int, table: bool = False, reps: int = 1) -> np.ndarray:
        """reps passes over each thread's contiguous share (timed baselines)."""
        out = np.empty(n, dtype=np.uint32)
        rc = self.lib.oracle_crc32c_fixed_mt_reps(buf.ctypes.data, stride, length, n,
                                                  out.ctypes.data, threads, int(table), reps)
        if rc != 0:
            raise RuntimeError("oracle_crc32c_fixed_mt failed")
        return out


class _Ref:
    """ctypes view of a reference-built library in oracle/_ref/."""

    def __init__(self, flavour: str) -> None:
        path = os.path.join(HERE, "_ref", f"libref_crc32c_{flavour}.so")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
        lib.ref_crc32c_extend.restype = ctypes.c_uint32
        lib.ref_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        lib.ref_crc32c_value.restype = ctypes.c_uint32
        lib.ref_crc32c_value.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        lib.ref_crc32c_mask.restype = ctypes.c_uint32
        lib.ref_crc32c_mask.argtypes = [ctypes.c_uint32]
        lib.ref_crc32c_unmask.restype = ctypes.c_uint32
        lib.ref_crc32c_unmask.argtypes = [ctypes.c_uint32]
        lib.ref_accelerated_crc32c.restype = ctypes.c_uint32
        lib.ref_accelerated_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        lib.ref_crc32c_fixed_mt.restype = ctypes.c_int
        lib.ref_crc32c_fixed_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_void_p, ctypes.c_int]
        lib.ref_crc32c_fixed_mt_reps.restype = ctypes.c_int
        lib.ref_crc32c_fixed_mt_reps.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64]
        if hasattr(lib, "ref_dbbench_crc32c"):
            lib.ref_dbbench_crc32c.restype = ctypes.c_uint64
            lib.ref_dbbench_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint32)]
        self.lib = lib
        self.path = path

    def dbbench_crc32c(self, fn_addr=None, total: int = 500 * 1048576) -> tuple:
        """db/db_bench.cc:729-746's crc32c loop (4 KiB Value() until `total`
        bytes) on this thread: the reference's Value (fn_addr None) or the C
        function at fn_addr with Value's signature.  (GiB/s, last crc)."""
        crc = ctypes.c_uint32(0)
        ns = self.lib.ref_dbbench_crc32c(fn_addr, total, ctypes.byref(crc))
        done = (total + 4095) // 4096 * 4096
        return done / (ns * 1e-9) / 2**30, crc.value

    def extend(self, init: int, data) -> int:
        b = bytes(data)
        return self.lib.ref_crc32c_extend(init & 0xFFFFFFFF, b, len(b))

    def extend_at(self, init: int, buf: np.ndarray, off: int, n: int) -> int:
        """Extend over buf[off:off+n] in place (keeps the true alignment)."""
        return self.lib.ref_crc32c_extend(init & 0xFFFFFFFF, buf.ctypes.data + off, n)

    def value(self, data) -> int:
        return self.extend(0, data)

    def mask(self, crc: int) -> int:
        return self.lib.ref_crc32c_mask(crc & 0xFFFFFFFF)

    def unmask(self, m: int) -> int:
        return self.lib.ref_crc32c_unmask(m & 0xFFFFFFFF)

    def fixed_mt(self, buf: np.ndarray, stride: int, length: int, n: int,
                 threads: int, reps: int = 1) -> np.ndarray:
        """reps passes over each thread's contiguous share (timed baselines)."""
        out = np.empty(n, dtype=np.uint32)
        rc = self.lib.ref_crc32c_fixed_mt_reps(buf.ctypes.data, stride, length, n,
                                               out.ctypes.data, threads, reps)
        if rc != 0:
            raise RuntimeError("ref_crc32c_fixed_mt failed")
        return out


_port = None
_refs: dict = {}


def port() -> _Port:
    global _port
    if _port is None:
        _port = _Port()
    return _port


def ref(flavour: str = "sse") -> _Ref:
    if flavour not in _refs:
        _refs[flavour] = _Ref(flavour)
    return _refs[flavour]


def ref_available(flavour: str = "sse") -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", f"libref_crc32c_{flavour}.so"))


class _RefFraming:
    """ctypes view of ``oracle/_ref/libref_framing.so`` (oracle/ref_framing.cc):
    the reference's own log::Writer, log::Reader and ReadBlock."""

    def __init__(self) -> None:
        self.path = os.path.join(HERE, "_ref", "libref_framing.so")
        lib = ctypes.CDLL(self.path, mode=os.RTLD_LOCAL)
        vp, u64, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t
        lib.ref_log_write.restype = ctypes.c_int
        lib.ref_log_write.argtypes = [vp, vp, sz, u64, vp, sz, vp]
        lib.ref_log_read.restype = ctypes.c_int
        lib.ref_log_read.argtypes = [vp, sz, ctypes.c_int, u64, vp, sz, vp]
        lib.ref_log_read_failing.restype = ctypes.c_int
        lib.ref_log_read_failing.argtypes = [vp, sz, ctypes.c_int, u64, u64, vp, sz, vp]
        lib.ref_read_block.restype = ctypes.c_int
        lib.ref_read_block.argtypes = [vp, sz, u64, u64, ctypes.c_char_p, sz]
        lib.ref_table_scan.restype = ctypes.c_int
        lib.ref_table_scan.argtypes = [vp, sz, vp, sz, vp]
        self.lib = lib

    def log_write(self, payloads: list[bytes], dest_length: int = 0) -> bytes:
        blob = b"".join(payloads) or b"\0"
        lens = np.array([len(p) for p in payloads] or [0], dtype=np.uint64)
        total = sum(len(p) for p in payloads)
        cap = total + 7 * (total // 8 + len(payloads) + 2) + 64
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        rc = self.lib.ref_log_write(blob, lens.ctypes.data, len(payloads), dest_length, out, cap, ctypes.byref(n))
        assert rc == 0, rc
        return out.raw[:n.value]

    def log_read(self, image: bytes, checksum: bool = True, initial_offset: int = 0) -> str:
        cap = 64 * (len(image) // 7 + 16) + 4096
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        rc = self.lib.ref_log_read(image or b"\0", len(image), int(checksum), initial_offset, out, cap,
                                   ctypes.byref(n))
        assert rc == 0, rc
        return out.raw[:n.value].decode()

    def log_read_failing(self, image: bytes, checksum: bool, initial_offset: int, fail_at: int) -> str:
        """log::Reader over a SequentialFile whose read covering byte fail_at fails."""
        cap = 64 * (len(image) // 7 + 16) + 4096
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        rc = self.lib.ref_log_read_failing(image or b"\0", len(image), int(checksum), initial_offset, fail_at, out,
                                           cap, ctypes.byref(n))
        assert rc == 0, rc
        return out.raw[:n.value].decode()

    def table_scan(self, image: bytes, cap: int = 1 << 20) -> str:
        """ref_table_scan trace; retried once with the exact size when `cap` is short."""
        n = ctypes.c_size_t(0)
        while True:
            out = ctypes.create_string_buffer(cap)
            rc = self.lib.ref_table_scan(image or b"\0", len(image), out, cap, ctypes.byref(n))
            if rc == -5 and n.value > cap:
                cap = n.value
                continue
            assert rc == 0, rc
            return out.raw[:n.value].decode()

    def read_block(self, image: bytes, offset: int, size: int) -> str:
        msg = ctypes.create_string_buffer(256)
        self.lib.ref_read_block(image or b"\0", len(image), offset, size, msg, 256)
        return msg.value.decode()


_ref_framing = None


def ref_framing() -> _RefFraming:
    global _ref_framing
    if _ref_framing is None:
        _ref_framing = _RefFraming()
    return _ref_framing


class _RefTable:
    """ctypes view of ``oracle/_ref/libref_table.so`` (oracle/ref_table.cc): the
    reference's own TableBuilder, writing to memory or through shims::TableFile."""

    def __init__(self, deferred: bool = False) -> None:
        self.path = os.path.join(HERE, "_ref", "libref_table_deferred.so" if deferred else "libref_table.so")
        lib = ctypes.CDLL(self.path, mode=os.RTLD_LOCAL)
        vp, sz, u64, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32
        lib.ref_table_build.restype = ctypes.c_int
        lib.ref_table_build.argtypes = [vp, vp, vp, sz, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int, u32, vp, sz,
                                        vp, vp, sz, vp, vp, vp]
        self.lib = lib

    def build(self, keys, values, block_size=4096, restart_interval=16, bloom_bits=0, via_shim=0,
              seal_flags=0):
        """(image bytes, block handles [(offset, size)] in write order -- via_shim
        only).  via_shim: 0 the reference's own file; 1 / 2 the shipped
        BatchingWritableFile sealing at Close / every ~5000 bytes; 3 its staged
        bytes before any seal (oracle/ref_table.cc).  self.seals: the seal
        batches of the last build; self.computed: the trailers that reached the
        adapter with a CRC the builder computed itself."""
        kv = b"".join(k + v for k, v in zip(keys, values)) or b"\0"
        kl = np.array([len(k) for k in keys] or [0], dtype=np.uint64)
        vl = np.array([len(v) for v in values] or [0], dtype=np.uint64)
        cap = len(kv) * 2 + 64 * len(keys) + (1 << 16)
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        hcap = 2 * (len(kv) // 16 + 64)
        hd = np.zeros(hcap, dtype=np.uint64)
        nh = ctypes.c_size_t(0)
        seals = ctypes.c_size_t(0)
        computed = ctypes.c_size_t(0)
        rc = self.lib.ref_table_build(kv, kl.ctypes.data, vl.ctypes.data, len(keys), block_size, restart_interval,
                                      bloom_bits, int(via_shim), seal_flags, out, cap, ctypes.byref(n),
                                      hd.ctypes.data, hcap, ctypes.byref(nh), ctypes.byref(seals),
                                      ctypes.byref(computed))
        assert rc == 0, rc
        self.seals = seals.value
        self.computed = computed.value
        hs = [(int(hd[2 * k]), int(hd[2 * k + 1])) for k in range(nh.value)]
        return out.raw[:n.value], hs


_ref_table = {}


def ref_table(deferred: bool = False):
    if deferred not in _ref_table:
        _ref_table[deferred] = _RefTable(deferred)
    return _ref_table[deferred]


def ref_table_available(deferred: bool = False) -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", "libref_table_deferred.so" if deferred else "libref_table.so"))


def ref_framing_available() -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", "libref_framing.so"))
