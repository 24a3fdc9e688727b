"""Whole-table verification (nvl_sstable_verify_table, include/nvl_framing.h;
nvl::shims::VerifyTable, include/nvl_leveldb_shims.h): footer -> index block
-> every data block, plus the metaindex and the blocks it points at, all
checked with ReadBlock's rules in one CRC batch.

Parity anchors:
* tests/golden/table_cases.json -- 330 table images (tests/table_cases.py:
  named cases for every Table::Open / ReadBlock / Block::Iter outcome plus
  seeded random ones) scanned by the REFERENCE's own Footer::DecodeFrom,
  ReadBlock and Block::Iter (table/format.cc, table/block.cc, built from
  /root/reference; oracle/ref_framing.cc:ref_table_scan).  The image is
  rebuilt from its spec and checked against the stored length and CRC first.
* live, where oracle/_ref/libref_framing.so exists: 200 further random tables.
* at size: a 10^5-block table (~400 MB) on the GPU -- every block verifies,
  then exactly the corrupted ones fail (size-independent property).

Each check runs with NVL_FRAMING_HOST (CPU suite) and on the GPU (marked gpu).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import table_cases as tc
from conftest import ROOT, gpu_present, load_golden

HOST = 0x100
GPU = 0x400  # NVL_FRAMING_GPU: force the GPU (flags = 0 picks by size)
NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.fixture(scope="module")
def L():
    from nvlevelz_amd import _lib
    return _lib


@pytest.fixture(scope="module")
def harness(L):
    path = os.path.join(NATIVE, "libshim_harness.so")
    # rebuilt when stale in the build container (the header is a dependency);
    # the GPU box uses the shipped .so unless it is missing
    if not os.path.exists(path) or os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", NATIVE, "libshim_harness.so"], check=True)
    lib = ctypes.CDLL(path)
    vp, sz, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32
    lib.shim_table_verify.restype = ctypes.c_int
    lib.shim_table_verify.argtypes = [vp, sz, u32, vp, sz, vp]
    lib.shim_table_read.restype = ctypes.c_int
    lib.shim_table_read.argtypes = [vp, sz, sz, u32, ctypes.c_int, vp, sz, vp, vp]
    return lib


def verify(L, img: bytes, flags: int):
    n = ctypes.c_size_t(0)
    st = ctypes.c_uint32(0)
    nb = ctypes.c_uint64(0)
    lib = L.lib
    # the size query (blocks = NULL) checks only the index and metaindex on the
    # host, and must still give the exact count and table status
    assert lib.nvl_sstable_verify_table(img, len(img), None, 0, ctypes.byref(n), ctypes.byref(st),
                                        ctypes.byref(nb), flags) == 0
    q_n, q_st = n.value, st.value
    arr = (L.TableBlock * max(n.value, 1))()
    assert lib.nvl_sstable_verify_table(img, len(img), arr, n.value, ctypes.byref(n), ctypes.byref(st),
                                        ctypes.byref(nb), flags) == 0
    assert (q_n, q_st) == (n.value, st.value)
    blocks = [(a.offset, a.size, a.role, a.verdict) for a in arr[:n.value]]
    assert nb.value == sum(b[3] != 0 for b in blocks)
    return st.value, blocks


def verify_dev(L, img: bytes):
    """nvl_sstable_verify_table_dev on a device copy of img (size query, then the list)."""
    import torch
    d = torch.frombuffer(bytearray(img or b"\0"), dtype=torch.uint8)[:len(img)].cuda()
    st_ = torch.cuda.current_stream().cuda_stream
    n = ctypes.c_size_t(0)
    st = ctypes.c_uint32(0)
    nb = ctypes.c_uint64(0)
    lib = L.lib
    assert lib.nvl_sstable_verify_table_dev(d.data_ptr(), len(img), None, 0, ctypes.byref(n), ctypes.byref(st),
                                            ctypes.byref(nb), st_) == 0
    q_n, q_st = n.value, st.value
    arr = (L.TableBlock * max(n.value, 1))()
    assert lib.nvl_sstable_verify_table_dev(d.data_ptr(), len(img), arr, n.value, ctypes.byref(n), ctypes.byref(st),
                                            ctypes.byref(nb), st_) == 0
    assert (q_n, q_st) == (n.value, st.value)
    blocks = [(a.offset, a.size, a.role, a.verdict) for a in arr[:n.value]]
    assert nb.value == sum(b[3] != 0 for b in blocks)
    return st.value, blocks


def via_header(harness, img: bytes, flags: int):
    cap = 64 * (len(img) // 8 + 16)
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    assert harness.shim_table_verify(img, len(img), flags, out, cap, ctypes.byref(n)) == 0
    lines = out.raw[:n.value].decode().splitlines()
    st, _ = map(int, lines[0].split())
    return st, [tuple(map(int, x.split())) for x in lines[1:]]


def via_reader(harness, img: bytes, flags: int, window: int, order: int):
    """nvl::shims::TableReader: Open + every data block read (forward or
    backward), window blocks checked per batch -> (status, blocks), batches."""
    cap = 64 * (len(img) // 8 + 16)
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    nb = ctypes.c_size_t(0)
    assert harness.shim_table_read(img, len(img), window, flags, order, out, cap, ctypes.byref(n),
                                   ctypes.byref(nb)) == 0
    lines = out.raw[:n.value].decode().splitlines()
    st, _ = map(int, lines[0].split())
    return (st, [tuple(map(int, x.split())) for x in lines[1:]]), nb.value


def _check_reader(harness, port, flags, every=10):
    """The batched table reader replays the 330 reference-scanned tables
    window by window: after reading every data block its verdicts equal the
    reference trace (the whole-table batch's), whatever the window and the
    read order; forward reads take ceil(data / window) batches (+ one for the
    meta blocks)."""
    cases = load_golden("table_cases")["cases"]
    for c in cases:
        if c["name"].startswith("random_") and int(c["name"][7:]) % every:
            continue
        img, _ = tc.build(port, c)
        want = tc.expected(c["trace"])
        nd = sum(1 for b in want[1] if b[2] == 3 and b[3] != 4)  # data blocks with a handle
        nm = sum(1 for b in want[1] if b[2] == 2 and b[3] != 4)
        for window in (1, 3, 17):
            for order in (0, 1):
                got, batches = via_reader(harness, img, flags, window, order)
                assert got == want, (c["name"], window, order)
                if order == 0:
                    assert batches <= (1 if nm else 0) + -(-nd // window), (c["name"], window, batches)


def test_table_reader_golden_host(harness, port):
    _check_reader(harness, port, HOST)


@pytest.mark.gpu
def test_table_reader_golden_gpu(harness, port):
    if not gpu_present():
        pytest.skip("no GPU")
    _check_reader(harness, port, GPU, every=30)


def _check_golden(L, harness, port, flags):
    cases = load_golden("table_cases")["cases"]
    assert len(cases) >= 300
    for c in cases:
        img, _ = tc.build(port, c)
        assert len(img) == c["image_len"] and port.value(img) == c["image_crc"], c["name"]
        want = tc.expected(c["trace"])
        assert verify(L, img, flags) == want, c["name"]
        if c["name"].startswith("random_") and int(c["name"][7:]) % 10:
            continue
        assert via_header(harness, img, flags) == want, c["name"]


def test_table_cases_golden_host(L, harness, port):
    _check_golden(L, harness, port, HOST)


@pytest.mark.gpu
def test_table_cases_golden_gpu(L, harness, port):
    if not gpu_present():
        pytest.skip("no GPU")
    _check_golden(L, harness, port, GPU)


@pytest.mark.gpu
def test_table_cases_golden_device_resident(L, port):
    """The same 330 reference traces through nvl_sstable_verify_table_dev on
    device copies of the images (the table already in HBM)."""
    if not gpu_present():
        pytest.skip("no GPU")
    for c in load_golden("table_cases")["cases"]:
        img, _ = tc.build(port, c)
        assert verify_dev(L, img) == tc.expected(c["trace"]), c["name"]


def _indexed_table(port, nblocks, interval, damage, seed):
    """A table of nblocks data blocks (1..2000 B, type 0/1), a filter block,
    the metaindex and an index block with the given restart interval (1: the
    TableBuilder form the GPU index parse reads; 2: prefix-compressed keys,
    which it hands to the sequential walk).  damage: a few index values that
    are no handle / point past the end, and flipped or retyped blocks."""
    rng = np.random.default_rng(seed)
    w = tc._Writer(port)
    pool = rng.integers(0, 256, 1 << 16, dtype=np.uint8).tobytes()
    ents = []
    for b in range(nblocks):
        n = int(rng.integers(1, 2000))
        s = int(rng.integers(0, len(pool) - n))
        h = w.raw(pool[s:s + n], int(rng.integers(0, 2)))
        key = b"user-key-%012d" % b + (b"~" * 150 if b % 97 == 5 else b"")  # some keys need 2-byte varints
        ents.append((key, tc.handle(*h)))
    filt = w.raw(pool[:777])
    meta_h = w.raw(tc.block([(b"filter.leveldb.BuiltinBloomFilter2", tc.handle(*filt))], 16))
    flips = []
    if damage:
        ents[5] = (ents[5][0], b"\xff")                               # not a BlockHandle
        ents[7] = (ents[7][0], tc.handle(len(w.img) + 1000, 10))      # past the end
        flips = sorted(set(int(x) for x in rng.integers(10, nblocks, 40)))
    idx = tc.block(ents, interval)
    index_h = w.raw(idx)
    foot = tc.handle(*meta_h) + tc.handle(*index_h)
    w.img += foot + bytes(40 - len(foot)) + tc.MAGIC.to_bytes(8, "little")
    img = bytearray(w.img)
    for b in flips:  # flip a content byte or the type byte of data block b
        off, n = tc._varint_handle(ents[b][1])
        img[off + (int(rng.integers(0, n)) if b % 3 else n)] ^= 0x40
    return bytes(img), len(flips)


@pytest.mark.gpu
@pytest.mark.parametrize("interval,damage", [(1, False), (1, True), (2, False), (2, True)])
def test_table_dev_index_parse_at_size(L, port, interval, damage):
    """A 20000-block table through nvl_sstable_verify_table_dev: the GPU
    index parse (interval 1) and the sequential fallback (interval 2) both
    give the host walk's list (NVL_FRAMING_HOST) exactly, clean and damaged."""
    if not gpu_present():
        pytest.skip("no GPU")
    img, nflip = _indexed_table(port, 20_000, interval, damage, 17 + interval)
    want = verify(L, img, HOST)
    got = verify_dev(L, img)
    assert got[0] == want[0] == 0
    assert len(got[1]) == len(want[1]) == 20_000 + 3
    bad = [i for i, (a, b) in enumerate(zip(got[1], want[1])) if a != b]
    assert not bad, (bad[:5], [got[1][i] for i in bad[:5]], [want[1][i] for i in bad[:5]])
    data_bad = sum(b[3] != 0 for b in want[1] if b[2] == 3)
    assert data_bad == (nflip + 2 if damage else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,nblocks", [("shuffled", 4000), ("overlapping", 4000), ("shuffled", 12000)])
def test_table_dev_out_of_order_index(L, port, mode, nblocks):
    """An index whose handles are NOT in file order (a crafted or corrupt
    table: keys in order, handles permuted, or every 5th pointing back into
    its predecessor): nvl_sstable_verify_table_dev runs its batch as ONE
    region-kernel launch up to 8192 slots (NVL_CRC32C_FLAG_REGION_SHAPED, the
    slots of a well-formed table are in file order), whose per-buffer path
    must still give every block the host walk's verdict; a larger table keeps
    the checked entry (its plan sends the batch to the batch kernels)."""
    if not gpu_present():
        pytest.skip("no GPU")
    import time
    rng = np.random.default_rng(23)
    w = tc._Writer(port)
    pool = rng.integers(0, 256, 1 << 16, dtype=np.uint8).tobytes()
    hs = []
    for b in range(nblocks):
        n = int(rng.integers(1, 4000))
        s = int(rng.integers(0, len(pool) - n))
        hs.append(w.raw(pool[s:s + n], int(rng.integers(0, 2))))
    if mode == "shuffled":
        hs = [hs[i] for i in rng.permutation(len(hs))]
    else:
        hs = [(o - (min(200, o) if i % 5 == 4 else 0), n) for i, (o, n) in enumerate(hs)]
    ents = [(b"user-key-%012d" % b, tc.handle(*h)) for b, h in enumerate(hs)]
    filt = w.raw(pool[:777])
    meta_h = w.raw(tc.block([(b"filter.leveldb.BuiltinBloomFilter2", tc.handle(*filt))], 16))
    index_h = w.raw(tc.block(ents, 1))
    foot = tc.handle(*meta_h) + tc.handle(*index_h)
    w.img += foot + bytes(40 - len(foot)) + tc.MAGIC.to_bytes(8, "little")
    img = bytes(w.img)
    want = verify(L, img, HOST)
    t0 = time.perf_counter()
    got = verify_dev(L, img)
    el = time.perf_counter() - t0
    assert got == want, [(a, b) for a, b in zip(got[1], want[1]) if a != b][:5]
    assert len(got[1]) == nblocks + 3
    if mode == "overlapping":
        assert sum(b[3] != 0 for b in want[1] if b[2] == 3) > 0  # the shifted handles fail their checks
    assert el < 5.0, el


def test_table_verify_dev_arguments(L):
    lib = L.lib
    n = ctypes.c_size_t(7)
    st = ctypes.c_uint32(9)
    assert lib.nvl_sstable_verify_table_dev(None, 5, None, 0, ctypes.byref(n), ctypes.byref(st), None, None) == L.EINVAL
    assert lib.nvl_sstable_verify_table_dev(None, 0, None, 0, None, ctypes.byref(st), None, None) == L.EINVAL
    # a file too short to be a table needs no device access
    assert lib.nvl_sstable_verify_table_dev(None, 0, None, 0, ctypes.byref(n), ctypes.byref(st), None, None) == 0
    assert (n.value, st.value) == (0, L.TABLE_TOO_SHORT)


def test_table_cases_vs_reference_live(L, port):
    import oracle
    if not oracle.ref_framing_available():
        pytest.skip("reference build (oracle/_ref) not present")
    rf = oracle.ref_framing()
    for spec in tc.random_cases(200, seed=99):
        img, _ = tc.build(port, spec)
        assert verify(L, img, HOST) == tc.expected(rf.table_scan(img)), spec["name"]


def test_table_verify_arguments(L):
    lib = L.lib
    n = ctypes.c_size_t(7)
    st = ctypes.c_uint32(9)
    assert lib.nvl_sstable_verify_table(None, 5, None, 0, ctypes.byref(n), ctypes.byref(st), None, HOST) == L.EINVAL
    assert lib.nvl_sstable_verify_table(b"", 0, None, 0, None, ctypes.byref(st), None, HOST) == L.EINVAL
    assert lib.nvl_sstable_verify_table(b"", 0, None, 0, ctypes.byref(n), ctypes.byref(st), None, HOST) == 0
    assert (n.value, st.value) == (0, L.TABLE_TOO_SHORT)


def test_table_verify_enospc(L, port):
    img, _ = tc.build(port, {"seed": 3, "nblocks": 5, "nmeta": 1})
    n = ctypes.c_size_t(0)
    st = ctypes.c_uint32(0)
    arr = (L.TableBlock * 3)()
    assert L.lib.nvl_sstable_verify_table(img, len(img), arr, 3, ctypes.byref(n), ctypes.byref(st), None,
                                          HOST) == L.ENOSPC
    assert n.value == 1 + 1 + 1 + 5


def _big_table(port, nblocks: int, block_bytes: int):
    """A table of nblocks data blocks of ~block_bytes (one key-value entry
    each), written with numpy: returns (image, data handles)."""
    ent_hdr = tc.varint(0) + tc.varint(16) + tc.varint(block_bytes - 30)
    vlen = block_bytes - 30
    body = len(ent_hdr) + 16 + vlen
    size = body + 8  # one restart + count
    stride = size + 5
    payload = port.fill(77, 0, nblocks * vlen).reshape(nblocks, vlen)
    img = np.zeros(nblocks * stride, dtype=np.uint8).reshape(nblocks, stride)
    img[:, :len(ent_hdr)] = np.frombuffer(ent_hdr, dtype=np.uint8)
    keys = np.array([list(b"k%015d" % i) for i in range(nblocks)], dtype=np.uint8)
    img[:, len(ent_hdr):len(ent_hdr) + 16] = keys
    img[:, len(ent_hdr) + 16:body] = payload
    img[:, body + 4] = 1  # num_restarts = 1 (restart[0] = 0)
    flat = img.reshape(-1)
    handles = np.stack([np.arange(nblocks, dtype=np.uint64) * stride, np.full(nblocks, size, np.uint64)], 1)
    # trailers: type 0 + Mask(Value(block | type)), sealed by the shim on the host
    buf = bytearray(flat.tobytes())
    return buf, handles, size


@pytest.mark.gpu
def test_table_verify_large_gpu(L, port):
    """10^5 data blocks of 4 KiB: all verify; then exactly the corrupted ones fail."""
    if not gpu_present():
        pytest.skip("no GPU")
    nblocks = 100_000
    buf, handles, size = _big_table(port, nblocks, 4096)
    h = np.ascontiguousarray(handles)
    cbuf = (ctypes.c_char * len(buf)).from_buffer(buf)
    assert L.lib.nvl_sstable_seal_trailers(cbuf, len(buf), h.ctypes.data, nblocks, GPU) == 0
    del cbuf  # release the export so the image can grow
    data_end = len(buf)
    w = tc._Writer(port)
    w.img = buf
    meta_h = w.raw(tc.block([], 16))
    index = tc.block([(b"k%015d" % i, tc.handle(int(o), int(s))) for i, (o, s) in enumerate(handles)], 1)
    index_h = w.raw(index)
    foot = tc.handle(*meta_h) + tc.handle(*index_h)
    w.img += foot + bytes(40 - len(foot)) + tc.MAGIC.to_bytes(8, "little")
    img = bytes(w.img)
    st, blocks = verify(L, img, GPU)
    assert st == 0 and len(blocks) == nblocks + 2
    assert all(b[3] == 0 for b in blocks)
    assert [b[:2] for b in blocks[2:]] == [(int(o), int(s)) for o, s in handles]
    rng = np.random.default_rng(11)
    bad_idx = sorted(set(int(x) for x in rng.integers(0, nblocks, 40)))
    mut = bytearray(img)
    for k in bad_idx:
        o = int(handles[k][0])
        mut[o + int(rng.integers(0, size))] ^= 1 << int(rng.integers(0, 8))
    assert data_end < len(mut)
    st, blocks = verify(L, bytes(mut), GPU)
    assert st == 0
    assert [i for i, b in enumerate(blocks[2:]) if b[3]] == bad_idx
    assert all(blocks[2 + k][3] == L.BLOCK_CHECKSUM_MISMATCH for k in bad_idx)
    # the table already in HBM: the same verdicts
    assert verify_dev(L, bytes(mut)) == (st, blocks)


# ---- Python view (nvlevelz_amd/framing.py) ---------------------------------

def _check_python_view(port, host):
    from nvlevelz_amd import framing
    for c in load_golden("table_cases")["cases"][:40]:
        img, _ = tc.build(port, c)
        st, want = tc.expected(c["trace"])
        rep = framing.verify_table(img, host=host)
        assert rep.status == st, c["name"]
        assert [(b.offset, b.size, b.verdict) for b in rep.blocks] == [w[:2] + (w[3],) for w in want], c["name"]
        if st == 0:
            assert rep.ok == all(w[3] == 0 for w in want)
        # the same blocks through verify_blocks
        if rep.blocks:
            v = framing.verify_blocks(img, [(b.offset, b.size) for b in rep.blocks if b.verdict != 4], host=host)
            assert list(v) == [b.verdict for b in rep.blocks if b.verdict != 4], c["name"]
    # a reference-derived status text
    img, _ = tc.build(port, {"seed": 5, "nblocks": 3, "nmeta": 1, "muts": [["magic"]]})
    assert framing.verify_table(img, host=host).status_text == "Corruption: not an sstable (bad magic number)"


def test_python_view_host(port):
    _check_python_view(port, True)


@pytest.mark.gpu
def test_python_view_gpu(port):
    if not gpu_present():
        pytest.skip("no GPU")
    _check_python_view(port, False)


@pytest.mark.skipif(gpu_present(), reason="checks the no-GPU behaviour")
def test_python_view_fails_loudly_without_gpu(port):
    from nvlevelz_amd import framing
    img, _ = tc.build(port, {"seed": 5, "nblocks": 3, "nmeta": 1})
    with pytest.raises(framing.FramingError):
        framing.verify_table(img, host=False)
