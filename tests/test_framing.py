"""The §8f call-site shims (include/nvl_framing.h, include/nvl_leveldb_shims.h):
log::Writer / log::Reader and SSTable block trailers with their CRCs batched.

Parity anchors:
* tests/golden/log_cases.json -- scenarios after db/log_test.cc plus seeded
  random ones (tests/framing_cases.py), each written and read by the
  REFERENCE's own db/log_writer.cc and db/log_reader.cc (oracle/ref_framing.cc,
  built from /root/reference): the image bytes (crc + length) and the full
  reader trace -- records returned, LastRecordOffset, every corruption report
  with its byte count and reason.
* tests/golden/framing.json -- block trailers / record headers computed with
  the reference's crc32c.
* live, where oracle/_ref/libref_framing.so exists: fresh random scenarios
  against the reference writer/reader, and every sealed or corrupted SSTable
  block through the reference's ReadBlock (table/format.cc:65-98).

Each check runs twice: NVL_FRAMING_HOST (host CRC; CPU suite) and the GPU
batch (marked gpu).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import framing_cases as fc
from conftest import ROOT, gpu_present, load_golden

NATIVE = os.path.join(ROOT, "tests", "native")
HOST = 0x100
GPU = 0x400  # NVL_FRAMING_GPU: force the GPU (flags = 0 picks by size)


@pytest.fixture(scope="module")
def shim():
    from nvlevelz_amd import _lib  # noqa: F401  (loads libnvl_crc32c.so first)
    path = os.path.join(NATIVE, "libshim_harness.so")
    if not os.path.exists(path) or os.path.isdir("/root/reference"):  # rebuilt when stale here
        subprocess.run(["make", "-s", "-C", NATIVE, "libshim_harness.so"], check=True)
    lib = ctypes.CDLL(path)
    vp, u64, sz, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32
    lib.shim_log_write.restype = ctypes.c_int
    lib.shim_log_write.argtypes = [vp, vp, sz, u64, u32, vp, sz, vp]
    lib.shim_log_read.restype = ctypes.c_int
    lib.shim_log_read.argtypes = [vp, sz, ctypes.c_int, u64, u32, vp, sz, vp]
    lib.shim_log_read_stream.restype = ctypes.c_int
    lib.shim_log_read_stream.argtypes = [vp, sz, ctypes.c_int, u64, u32, sz, u64, vp, sz, vp, vp]
    return lib


@pytest.fixture(scope="module")
def L():
    from nvlevelz_amd import _lib
    return _lib


def _writer(shim, flags):
    def w(payloads, dest_length):
        blob = b"".join(payloads) or b"\0"
        lens = np.array([len(p) for p in payloads] or [0], dtype=np.uint64)
        total = sum(len(p) for p in payloads)
        cap = total + 7 * (total // 8 + len(payloads) + 2) + 64
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        rc = shim.shim_log_write(blob, lens.ctypes.data, len(payloads), dest_length, flags, out, cap,
                                 ctypes.byref(n))
        assert rc == 0, rc
        return out.raw[:n.value]
    return w


def _reader(shim, flags):
    def r(image, checksum, initial_offset):
        cap = 64 * (len(image) // 7 + 16) + 4096
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        rc = shim.shim_log_read(image or b"\0", len(image), int(checksum), initial_offset, flags, out, cap,
                                ctypes.byref(n))
        assert rc == 0, rc
        return out.raw[:n.value].decode()
    return r


NO_FAIL = (1 << 64) - 1


def _stream_reader(shim, flags, window_blocks, fail_at=NO_FAIL):
    """The streaming shims::LogReader (a LogSource read window_blocks pieces at a
    time); returns (trace, number of source reads)."""
    def r(image, checksum, initial_offset):
        cap = 64 * (len(image) // 7 + 16) + 4096
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        reads = ctypes.c_size_t(0)
        rc = shim.shim_log_read_stream(image or b"\0", len(image), int(checksum), initial_offset, flags,
                                       window_blocks, fail_at, out, cap, ctypes.byref(n), ctypes.byref(reads))
        assert rc == 0, rc
        return out.raw[:n.value].decode(), reads.value
    return r


def _check_log_fixtures(shim, port, flags):
    cases = load_golden("log_cases")["cases"]
    assert len(cases) >= 300
    w, r = _writer(shim, flags), _reader(shim, flags)
    for c in cases:
        img = fc.write_image(port, c, w)
        assert (len(img), port.value(img)) == (c["image_len"], c["image_crc"]), c["name"]
        bad = fc.mutate(port, img, c["mutations"])
        assert (len(bad), port.value(bad)) == (c["read_len"], c["read_crc"]), c["name"]
        trace = r(bad, c["checksum"], c["initial_offset"])
        if "trace" in c:
            assert trace == c["trace"], c["name"]
        else:
            assert (port.value(trace.encode()), trace.count("\n")) == (c["trace_crc"], c["trace_lines"]), c["name"]


def test_log_fixtures_host(shim, port):
    _check_log_fixtures(shim, port, HOST)


@pytest.mark.gpu
def test_log_fixtures_gpu(shim, port):
    if not gpu_present():
        pytest.skip("no GPU")
    _check_log_fixtures(shim, port, GPU)


def _check_log_fixtures_streamed(shim, port, flags, windows):
    """The 334 log fixtures through the streaming reader, fed in windows of
    1, 3 and 17 blocks: the same trace as the whole-image reader (and as the
    reference, which the fixture traces come from), with ceil(len / window)
    + 1 reads at most (db/log_reader.cc:199-218 reads kBlockSize at a time)."""
    cases = load_golden("log_cases")["cases"]
    w = _writer(shim, flags)
    for wb in windows:
        r = _stream_reader(shim, flags, wb)
        for c in cases:
            bad = fc.mutate(port, fc.write_image(port, c, w), c["mutations"])
            trace, reads = r(bad, c["checksum"], c["initial_offset"])
            if "trace" in c:
                assert trace == c["trace"], (wb, c["name"])
            else:
                assert (port.value(trace.encode()), trace.count("\n")) == (c["trace_crc"], c["trace_lines"]), \
                    (wb, c["name"])
            assert reads <= len(bad) // (wb * 32768) + 2, (wb, c["name"], reads)


def test_log_fixtures_streamed_host(shim, port):
    _check_log_fixtures_streamed(shim, port, HOST, (1, 3, 17))


@pytest.mark.gpu
def test_log_fixtures_streamed_gpu(shim, port):
    if not gpu_present():
        pytest.skip("no GPU")
    _check_log_fixtures_streamed(shim, port, GPU, (1, 3, 17))


def test_log_stream_read_errors_vs_reference_live(shim, port):
    """A read that fails part way (IOError with the bytes before the failure):
    the streaming reader reports the reference's ReportDrop(kBlockSize,
    status) (db/log_reader.cc:205-211) -- same trace as the reference's
    log::Reader over the same failing SequentialFile, for failures at block
    boundaries, inside blocks, before/after initial_offset, and in windows of
    1, 3 and 17 blocks; a skip past the end (initial_offset beyond the file)
    too."""
    import oracle
    if not oracle.ref_framing_available():
        pytest.skip("reference framing harness not built")
    rf = oracle.ref_framing()
    w = _writer(shim, HOST)
    rng = np.random.default_rng(2024)
    specs = fc.random_cases(40, seed=4242)
    n = 0
    for spec in specs:
        img = fc.write_image(port, spec, w)
        muts, io = fc.resolve(port, spec, img)
        bad = fc.mutate(port, img, muts)
        L = len(bad)
        fails = {NO_FAIL, 0, L // 2, max(0, L - 1)}
        for k in range(1, L // 32768 + 1):
            fails |= {32768 * k, 32768 * k - 1, 32768 * k + 7}
        fails |= {int(x) for x in rng.integers(0, L + 1, 3)}
        for fa in sorted(fails):
            want = rf.log_read_failing(bad, spec["checksum"], io, min(fa, (1 << 64) - 1))
            for wb in (1, 3, 17):
                got, _ = _stream_reader(shim, HOST, wb, fa)(bad, spec["checksum"], io)
                assert got == want, (spec["name"], fa, wb)
                n += 1
        far = L + 5 * 32768  # initial_offset past the end: Skip fails (never reported), no records
        got, _ = _stream_reader(shim, HOST, 3)(bad, spec["checksum"], far)
        assert got == rf.log_read_failing(bad, spec["checksum"], far, NO_FAIL), spec["name"]
    assert n > 500


def test_log_vs_reference_live(shim, port):
    import oracle
    if not oracle.ref_framing_available():
        pytest.skip("reference framing harness not built")
    rf = oracle.ref_framing()
    w, r = _writer(shim, HOST), _reader(shim, HOST)
    for spec in fc.random_cases(150, seed=777):
        ref_img = fc.write_image(port, spec, rf.log_write)
        assert fc.write_image(port, spec, w) == ref_img, spec["name"]
        muts, io = fc.resolve(port, spec, ref_img)
        bad = fc.mutate(port, ref_img, muts)
        assert r(bad, spec["checksum"], io) == rf.log_read(bad, spec["checksum"], io), spec["name"]


def test_log_scan_arguments(L):
    ev = (L.LogEvent * 4)()
    n = ctypes.c_size_t(0)
    assert L.lib.nvl_log_scan(None, 0, 5, 1, ev, 4, ctypes.byref(n), HOST) == L.EINVAL  # start not block-aligned
    assert L.lib.nvl_log_scan(None, 0, 0, 1, ev, 4, None, HOST) == L.EINVAL
    assert L.lib.nvl_log_scan(None, 0, 0, 1, ev, 4, ctypes.byref(n), HOST) == L.OK
    assert n.value == 1 and ev[0].kind == L.LOG_EOF
    img = bytes(7) + b"abc"  # a zero record, then garbage
    assert L.lib.nvl_log_scan(img, len(img), 0, 1, None, 0, ctypes.byref(n), HOST) == L.OK and n.value == 2  # ZERO, EOF
    assert L.lib.nvl_log_scan(img, len(img), 0, 1, ev, 1, ctypes.byref(n), HOST) == L.ENOSPC


def test_log_record_headers_golden(L, port):
    """framing.json log records: header CRC of type | payload, via nvl_log_seal."""
    for rec in load_golden("framing")["log_records"]:
        payload = port.fill(int(rec["seed"]), 0, int(rec["len"])).tobytes()
        n = len(payload)
        img = bytearray(b"\0\0\0\0" + bytes([n & 0xFF, n >> 8, int(rec["type"])]) + payload)
        off = np.array([0], dtype=np.uint64)
        assert L.lib.nvl_log_seal((ctypes.c_char * len(img)).from_buffer(img), len(img), off.ctypes.data, 1,
                                  HOST) == 0
        assert int.from_bytes(img[:4], "little") == int(rec["masked"])


# ---------------------------------------------------------------- SSTable --

def _table(port, seed, nblocks):
    """A table-file-like image: blocks of random size and type, 5-byte trailers
    (type, zero CRC), random filler between some of them (index/footer bytes)."""
    rng = np.random.default_rng(seed)
    img = bytearray()
    handles = []
    for i in range(nblocks):
        if rng.random() < 0.2:
            img += port.fill(seed * 1000 + i, 7, int(rng.integers(1, 64))).tobytes()
        n = int(rng.choice([0, 1, 3, 4, 5, 17, 64, 4096, 4100, int(rng.integers(0, 9000))]))
        handles.append((len(img), n))
        img += port.fill(seed * 1000 + i, 0, n).tobytes()
        img += bytes([int(rng.choice([0, 0, 0, 1]))]) + bytes(4)
    return img, np.array(handles, dtype=np.uint64).reshape(-1, 2)


def _seal(L, img, handles, flags):
    buf = (ctypes.c_char * len(img)).from_buffer(img)
    h = np.ascontiguousarray(handles, dtype=np.uint64)
    return L.lib.nvl_sstable_seal_trailers(buf, len(img), h.ctypes.data, len(h), flags)


def _verify(L, img, handles, flags):
    h = np.ascontiguousarray(handles, dtype=np.uint64)
    v = np.zeros(len(h), dtype=np.uint8)
    nb = ctypes.c_uint64(0)
    rc = L.lib.nvl_sstable_verify_blocks(bytes(img), len(img), h.ctypes.data, len(h), v.ctypes.data,
                                         ctypes.byref(nb), flags)
    assert rc == 0, rc
    assert nb.value == int((v != 0).sum())
    return v


def _ref_verdict(msg, block_type):
    """ReadBlock's Status text -> NVL_BLOCK_* (type 1 blocks are then decompressed
    by ReadBlock; without snappy that fails, and it is out of the shim's scope)."""
    if msg == "" or (block_type == 1 and msg == "Corruption: corrupted compressed block contents"):
        return 0
    return {"Corruption: truncated block read": 1, "Corruption: block checksum mismatch": 2,
            "Corruption: bad block type": 3}[msg]


def _check_sstable(L, port, flags):
    import oracle
    rf = oracle.ref_framing() if oracle.ref_framing_available() else None
    for seed in range(1, 9):
        img, hs = _table(port, seed, 60)
        assert _seal(L, img, hs, flags) == 0
        for off, n in hs:  # table_builder.cc:185-187
            off, n = int(off), int(n)
            want = port.mask(port.value(bytes(img[off:off + n + 1])))
            assert int.from_bytes(img[off + n + 1:off + n + 5], "little") == want
        assert not _verify(L, img, hs, flags).any()
        rng = np.random.default_rng(seed)
        bad = bytearray(img)
        for _ in range(12):  # corrupt contents, type bytes, stored CRCs
            k = int(rng.integers(0, len(hs)))
            off, n = int(hs[k][0]), int(hs[k][1])
            what = rng.integers(0, 3)
            if what == 0 and n:
                bad[off + int(rng.integers(0, n))] ^= 1 << int(rng.integers(0, 8))
            elif what == 1:
                bad[off + n] = int(rng.integers(2, 256))
                bad[off + n + 1:off + n + 5] = int(port.mask(port.value(bytes(bad[off:off + n + 1])))).to_bytes(
                    4, "little")
            else:
                bad[off + n + 1 + int(rng.integers(0, 4))] ^= 0x40
        hs2 = np.concatenate([hs, np.array([[len(bad) - 3, 0], [len(bad) + 10, 5]], dtype=np.uint64)])
        v = _verify(L, bad, hs2, flags)
        assert v[-2] == 1 and v[-1] == 1  # truncated
        for k in range(len(hs)):
            off, n = int(hs[k][0]), int(hs[k][1])
            crc_ok = port.value(bytes(bad[off:off + n + 1])) == port.unmask(
                int.from_bytes(bad[off + n + 1:off + n + 5], "little"))
            want = 2 if not crc_ok else (3 if bad[off + n] > 1 else 0)
            assert v[k] == want, (seed, k)
            if rf is not None:
                assert _ref_verdict(rf.read_block(bytes(bad), off, n), bad[off + n]) == want, (seed, k)


def test_sstable_seal_verify_host(L, port):
    _check_sstable(L, port, HOST)


@pytest.mark.gpu
def test_sstable_seal_verify_gpu(L, port):
    if not gpu_present():
        pytest.skip("no GPU")
    _check_sstable(L, port, GPU)


def test_sstable_trailers_golden(L):
    """framing.json SSTable blocks: trailer = Mask(Value(block | type)) from the reference."""
    for b in load_golden("framing")["sstable_blocks"]:
        data = bytes.fromhex(b["hex"])
        img = bytearray(data + bytes([int(b["type"])]) + bytes(4))
        assert _seal(L, img, np.array([[0, len(data)]], dtype=np.uint64), HOST) == 0
        assert int.from_bytes(img[-4:], "little") == int(b["masked"])


def test_engine_policy_follows_host_tier():
    """the default crossover follows the host CRC tier -- 64 MiB
    over the AVX-512 folding tier, 16 MiB over SSE4.2 (its measured ~17 MiB
    crossover) and slice-by-8."""
    code = ("import sys; sys.path.insert(0, %r); from nvlevelz_amd import _lib; "
            "print(_lib.lib.nvl_crc32c_host_impl().decode(), _lib.lib.nvl_framing_gpu_min_bytes())" % ROOT)
    env = {k: v for k, v in os.environ.items() if k not in ("NVL_FRAMING_GPU_MIN_BYTES", "NVL_CRC32C_HOST")}
    for cap in ("sse", "table", None):
        e = dict(env, NVL_CRC32C_HOST=cap) if cap else env
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, env=e)
        assert r.returncode == 0, r.stderr
        impl, m = r.stdout.rsplit(None, 1)
        want = (64 << 20) if impl.startswith("avx512") else (16 << 20)
        assert int(m) == want, (cap, impl, m)


@pytest.mark.skipif(gpu_present(), reason="checks the no-GPU behaviour")
def test_device_mode_fails_loudly_without_gpu(L):
    img = bytearray(b"abc" + bytes(5))
    h = np.array([[0, 3]], dtype=np.uint64)
    assert _seal(L, img, h, GPU) in (L.ENODEV, L.EHIP)
    assert img[-4:] == bytes(4)  # nothing written
    n = ctypes.c_size_t(0)
    log = bytes(7)
    log = b"\x01\x02\x03\x04\x01\x00\x01x"
    assert L.lib.nvl_log_scan(log, len(log), 0, 1, None, 0, ctypes.byref(n), GPU) in (L.ENODEV, L.EHIP)


def test_python_view_log(port):
    """nvlevelz_amd.framing.log_seal / log_scan (host CRC): sealed headers match
    the reference's Mask(Value(type | payload)), a flipped payload byte is a
    checksum event that drops the rest of its block (log_reader.cc:254-267)."""
    from nvlevelz_amd import framing
    img, hdrs = bytearray(), []
    for k, n in enumerate([10, 300, 0, 5000]):
        hdrs.append(len(img))
        img += bytes(4) + bytes([n & 0xFF, n >> 8, 1]) + port.fill(k, 0, n).tobytes()
    framing.log_seal(img, hdrs, host=True)
    for h in hdrs:
        n = img[h + 4] | (img[h + 5] << 8)
        assert int.from_bytes(img[h:h + 4], "little") == port.mask(port.value(bytes(img[h + 6:h + 7 + n])))
    ev = framing.log_scan(bytes(img), host=True)
    assert [e[0] for e in ev] == ["record"] * 4 + ["eof"]
    assert [e[1] for e in ev[:4]] == hdrs
    bad = bytearray(img)
    bad[hdrs[1] + 9] ^= 1
    ev = framing.log_scan(bytes(bad), host=True)
    assert [e[0] for e in ev] == ["record", "checksum mismatch", "eof"]


def test_engine_policy(L):
    """flags = 0 picks the engine by the checksummed bytes of a host-resident
    call (the measured crossover); NVL_FRAMING_HOST / _GPU force one;
    both at once is an argument error."""
    lib = L.lib
    m = lib.nvl_framing_gpu_min_bytes()
    assert m > 0
    for b in (0, 1, m - 1):
        assert lib.nvl_framing_uses_gpu(b, 0) == 0
    for b in (m, m + 1, 1 << 40):
        assert lib.nvl_framing_uses_gpu(b, 0) == 1
    for b in (0, 1 << 40):
        assert lib.nvl_framing_uses_gpu(b, HOST) == 0
        assert lib.nvl_framing_uses_gpu(b, GPU) == 1
        assert lib.nvl_framing_uses_gpu(b, HOST | GPU) == L.EINVAL
    img = bytearray(b"abc" + bytes(5))
    h = np.array([[0, 3]], dtype=np.uint64)
    assert _seal(L, img, h, HOST | GPU) == L.EINVAL and img[-4:] == bytes(4)


def test_engine_policy_env_override():
    code = ("import sys; sys.path.insert(0, %r); from nvlevelz_amd import _lib; "
            "print(_lib.lib.nvl_framing_gpu_min_bytes(), _lib.lib.nvl_framing_uses_gpu(5000, 0), "
            "_lib.lib.nvl_framing_uses_gpu(4999, 0))" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, NVL_FRAMING_GPU_MIN_BYTES="5000"))
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["5000", "1", "0"]


@pytest.mark.skipif(gpu_present(), reason="checks the no-GPU behaviour")
def test_engine_policy_without_gpu(L, port):
    """No GPU: a small host-resident call takes the host CRC by policy and is
    right; a call the policy sends to the GPU fails loudly (no fallback)."""
    blocks = [port.fill(3 + k, 0, 1000).tobytes() for k in range(4)]
    img, hs = bytearray(), []
    for b in blocks:
        hs.append((len(img), len(b)))
        img += b + b"\0" + bytes(4)
    h = np.array(hs, dtype=np.uint64)
    assert _seal(L, img, h, 0) == L.OK
    for (o, n) in hs:
        assert int.from_bytes(img[o + n + 1:o + n + 5], "little") == port.mask(port.value(bytes(img[o:o + n + 1])))
    m = L.lib.nvl_framing_gpu_min_bytes()
    big = bytearray(m + 5)
    hb = np.array([[0, m]], dtype=np.uint64)
    assert _seal(L, big, hb, 0) in (L.ENODEV, L.EHIP)
    assert big[-4:] == bytes(4)
