"""GPU parity of the region path (nvl_crc32c_region_dev): the
region is checksummed in its own page-aligned 4 KiB chunks and every buffer
is derived from chunk raws, the events' masked butterflies (Qe) and the
fold kernel's piece-prefix re-reads (model: tests/kernel_model.py
region_batch).

Cases: BASELINE config 3 at full size (packed, unaligned starts, 512 B - 64
KiB); the SSTable shapes `r` (block | type, 3364..4109 B, 4-byte gaps) and
`v` (4097 B); starts and ends at every offset of a 128-byte window (every
lane, granule and dword position around a piece boundary) and around chunk
boundaries; 0..3-byte and sub-64-byte buffers (checksummed whole by the fold
kernel); buffers spanning many chunks; a region that does not start on a
page; per-buffer inits and Mask; and the layouts the fast path does not take
(unsorted, overlapping, a buffer outside the region), which must still be
right, followed by a sorted call on the same stream (the flag is reset).
Every CRC is compared with the oracle."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nvlevelz_amd import crc32c
    d = torch.device("cuda:0")
    torch.cuda.set_device(d)
    crc32c.init(0)
    return d


@pytest.fixture(scope="module")
def C():
    from nvlevelz_amd import crc32c
    return crc32c


def _u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def _t64(a, dev):
    return torch.from_numpy(np.asarray(a, dtype=np.int64)).to(dev)


def _region(C, dev, buf, offs, lens, init=0, mask=False, ws=None):
    if not isinstance(init, int):
        init = torch.from_numpy(np.asarray(init, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    return _u32(C.extend_region(buf, _t64(offs, dev), _t64(lens, dev), init, mask=mask, workspace=ws))


def _check(C, dev, port, host, buf, offs, lens, seed, mask_too=True):
    rng = np.random.default_rng(seed)
    n = len(offs)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    want = port.varlen(host, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint64), inits)
    got = _region(C, dev, buf, offs, lens, inits)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:10], np.asarray(lens)[bad[:10]], np.asarray(offs)[bad[:10]])
    if mask_too:
        want0 = port.varlen(host, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint64))
        got = _region(C, dev, buf, offs, lens, 0, mask=True)
        assert np.array_equal(got, np.array([port.mask(int(x)) for x in want0], dtype=np.uint32))


def _packed(port, lens, gap, seed, lead=0, tail=64):
    lens = np.asarray(lens, dtype=np.int64)
    offs = (lead + np.cumsum(lens + gap) - lens - gap).astype(np.int64)
    total = int(offs[-1] + lens[-1]) + tail if len(lens) else tail
    host = port.fill(seed, 0, total)
    return offs, host


def test_config3_full_region(dev, C, port):
    """BASELINE config 3 (1 GiB packed) through the region path: golden
    first/last CRCs and digest, and every CRC against the oracle."""
    g = load_golden("configs")["cfg3"]
    lens = port.cfg3_lengths(g["len_seed"], g["total"]).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    total = g["total"]
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, total // 8, 8, g["seed"])
    got = _region(C, dev, buf, offs, lens)
    assert [int(x) for x in got[:8]] == g["crc_first"]
    assert int(got[-1]) == g["crc_last"]
    assert port.digest(got) == g["digest"]
    want = port.varlen(buf.cpu().numpy(), offs.astype(np.uint64), lens.astype(np.uint64))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n", [1, 7, 390, 3000, 100_000])
def test_region_sstable_block_shape(dev, C, port, n):
    """block | type of data blocks at block_size 4096 (`r`): 4-byte gaps."""
    rng = np.random.default_rng(n)
    lens = rng.integers(3364, 4110, n)
    offs, host = _packed(port, lens, 4, 0x5B + n, lead=int(rng.integers(0, 16)))
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, n)


@pytest.mark.parametrize("gap", [4, 0, 1, 11])
def test_region_verify_shape_4097(dev, C, port, gap):
    """4096-byte blocks + type byte (`v`)."""
    n = 20_000
    lens = np.full(n, 4097)
    offs, host = _packed(port, lens, gap, 0x4097 + gap, lead=gap)
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, gap)


@pytest.mark.parametrize("lead", [0, 1, 3, 63, 64, 4093])
def test_region_every_offset(dev, C, port, lead):
    """Buffers whose starts and ends walk every byte of a 128-byte window
    around a piece boundary and of the chunk boundary (each buffer is 4096+k
    or 64+k bytes, so consecutive boundaries step by one byte)."""
    lens = []
    for k in range(130):
        lens += [4096 + k, 64 + k, 63 - (k % 64), 8192 + 3 * k]
    offs, host = _packed(port, lens, 0, 0xE0 + lead, lead=lead)
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, lead)


def test_region_tiny_and_mixed(dev, C, port):
    """0..3-byte, sub-64-byte and 64-byte buffers between big ones, gaps of
    0..70 bytes, a buffer ending exactly on a chunk end and one starting on a
    chunk start, multi-chunk buffers (up to 300 KB)."""
    rng = np.random.default_rng(11)
    lens, gaps = [], []
    for _ in range(3000):
        r = rng.random()
        lens.append(int(rng.integers(0, 4)) if r < 0.2 else int(rng.integers(4, 64)) if r < 0.35 else
                    64 if r < 0.4 else int(rng.integers(65, 9000)) if r < 0.97 else int(rng.integers(9000, 300_000)))
        gaps.append(int(rng.integers(0, 71)) if rng.random() < 0.5 else 0)
    lens = np.array(lens, dtype=np.int64)
    gaps = np.array(gaps, dtype=np.int64)
    offs = (np.cumsum(lens + gaps) - lens).astype(np.int64)
    # snap one end and one start onto chunk boundaries
    host = port.fill(0x7171, 0, int(offs[-1] + lens[-1]) + 4096)
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, 11)
    offs2 = np.array([4096 - 100, 4096, 8192 + 17, 3 * 4096], dtype=np.int64)
    lens2 = np.array([100, 4096 + 17, 4096 - 17, 4096], dtype=np.int64)
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs2, lens2, 12)


@pytest.mark.parametrize("shaped", [False, True])
def test_region_long_buffers(dev, C, port, shaped):
    """Buffers of three chunks and more: the fold's chain of up to four
    chunks per step (every remainder 1..4, chunk-aligned ends) and x^(8L)
    for T -- from the tables up to 1 MiB, through x^(2^k) beyond (the
    region kernel runs such buffers only under NVL_CRC32C_FLAG_REGION_SHAPED:
    the checked entry routes buffers over 128 KiB to the batch kernels)."""
    lens = [8193, 8192 + 4097, 4 * 4096, 5 * 4096 + 1, 6 * 4096 - 1, 7 * 4096, 9 * 4096 + 100, 65543, 131072,
            (1 << 20) - 1, (1 << 20) + 5, 3 * (1 << 20) + 4097, 130000, 3, 4097, 64]
    rng = np.random.default_rng(77)
    gaps = rng.integers(0, 9, len(lens))
    offs, host = _packed(port, lens, 0, 0x10E6, lead=5)
    offs = offs + np.cumsum(gaps) - gaps
    host = port.fill(0x10E6, 0, int(offs[-1] + lens[-1]) + 64)
    buf = torch.from_numpy(host).to(dev)
    inits = rng.integers(0, 2**32, size=len(lens), dtype=np.uint64).astype(np.uint32)
    want = port.varlen(host, offs.astype(np.uint64), np.asarray(lens, dtype=np.uint64), inits)
    it = torch.from_numpy(inits.view(np.int32)).to(dev)
    got = _u32(C.extend_region(buf, _t64(offs, dev), _t64(lens, dev), it, shaped=shaped))
    assert np.array_equal(got, want), np.nonzero(got != want)[0]


@pytest.mark.parametrize("skew", [1, 5, 2049])
def test_region_unaligned_region_pointer(dev, C, port, skew):
    """The region tensor starts `skew` bytes into an allocation: the chunk
    grid is page-aligned below it and offsets are region-relative."""
    rng = np.random.default_rng(skew)
    lens = rng.integers(100, 12000, 2000)
    offs, host = _packed(port, lens, 3, 0xA1 + skew, lead=0, tail=0)
    full = np.zeros(len(host) + skew + 64, dtype=np.uint8)
    full[skew:skew + len(host)] = host
    t = torch.from_numpy(full).to(dev)
    region = t[skew:skew + len(host)]
    _check(C, dev, port, host, region, offs, lens, skew)


def test_region_other_layouts_are_correct(dev, C, port):
    """Unsorted, overlapping and out-of-region batches through the checked
    entry: the plan sends them to the batch kernels, correct; a
    sorted call on the same stream afterwards takes the region path and is
    correct again.  (The region kernel's own per-buffer fallback for such
    batches is test_region_shaped_flag_on_other_layouts.)"""
    rng = np.random.default_rng(5)
    host = port.fill(0x515, 0, 200_000)
    buf = torch.from_numpy(host).to(dev)
    n = 500
    lens = rng.integers(0, 6000, n)
    offs = rng.integers(0, len(host) - 6000, n)
    _check(C, dev, port, host, buf, offs, lens, 1, mask_too=False)  # unsorted and overlapping
    lens_s = rng.integers(64, 300, n)
    offs_s, _ = _packed(port, lens_s, 0, 0, lead=0)
    _check(C, dev, port, host, buf, offs_s, lens_s, 2)  # sorted, after the flagged call
    # one buffer past the region's end (still inside the allocation)
    region = buf[:100_000]
    offs_o = np.array([10, 5000, 99_000], dtype=np.int64)
    lens_o = np.array([4000, 90_000, 5000], dtype=np.int64)
    want = port.varlen(host, offs_o.astype(np.uint64), lens_o.astype(np.uint64))
    got = _region(C, dev, region, offs_o, lens_o)
    assert np.array_equal(got, want)
    _check(C, dev, port, host, buf, offs_s, lens_s, 3)


def test_region_shaped_flag_on_other_layouts(dev, C, port):
    """NVL_CRC32C_FLAG_REGION_SHAPED on batches that are NOT region-shaped
    (ADVICE r05): the one-launch region kernel runs them anyway, and the
    header promises correct results -- buffers whose event records are
    missing (unsorted, overlapping), lie outside the region, or are longer
    than NVL_CRC32C_REGION_MAX_LEN (re-streamed halos) go through the
    kernel's per-buffer fallback (fold_in's inside rule, the records'
    buffer-index check).  Calls alternate with sorted ones on ONE caller
    workspace, so every stale record of the previous call is present."""
    rng = np.random.default_rng(77)
    host = port.fill(0x5A9E, 0, 900_000)
    buf = torch.from_numpy(host).to(dev)
    region = buf[:600_000]
    n = 400
    wsb = max(C.region_workspace_bytes(900_000, 3 * n), C.region_workspace_bytes(600_000, 3 * n))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    lens_s = rng.integers(64, 1500, n)
    offs_s, _ = _packed(port, lens_s, 3, 0, lead=11)

    def run(r, offs, lens, name):
        offs, lens = np.asarray(offs, dtype=np.int64), np.asarray(lens, dtype=np.int64)
        inits = rng.integers(0, 2**32, size=len(offs), dtype=np.uint64).astype(np.uint32)
        want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), inits)
        it = torch.from_numpy(inits.view(np.int32)).to(dev)
        got = _u32(C.extend_region(r, _t64(offs, dev), _t64(lens, dev), it, workspace=ws, shaped=True))
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (name, bad[:8], offs[bad[:8]], lens[bad[:8]])

    lens_u = rng.integers(0, 6000, n)
    offs_u = rng.integers(0, 600_000 - 6000, n)
    run(region, offs_u, lens_u, "unsorted + overlapping")
    run(region, offs_s, lens_s, "sorted after unsorted")
    perm = rng.permutation(n)
    run(region, offs_s[perm], lens_s[perm], "sorted blocks shuffled")
    run(region, offs_s, lens_s, "sorted after shuffled")
    ov = offs_s.copy()
    ov[1::7] -= 40  # every 7th buffer starts inside its predecessor
    run(region, ov, lens_s, "overlapping neighbours")
    # buffers past the region's end (inside the allocation: caller memory)
    offs_o = np.concatenate([offs_s[:50], [590_000, 599_990, 650_000]])
    lens_o = np.concatenate([lens_s[:50], [20_000, 100, 5000]])
    run(region, offs_o, lens_o, "outside the region")
    # buffers over 128 KiB among short ones, sorted (halos spanning many
    # workgroups' ranges, folded serially by their owner)
    lens_l = np.array([100, 140_000, 3000, 300_000, 17, 131_073, 131_072, 4096], dtype=np.int64)
    offs_l, _ = _packed(port, lens_l, 9, 0, lead=5)
    run(buf, offs_l, lens_l, "buffers over NVL_CRC32C_REGION_MAX_LEN")
    run(region, offs_s, lens_s, "sorted after long buffers")


def test_region_many_small_and_windows(dev, C, port):
    """Buffers of 64..200 bytes: up to 64 events per chunk and units whose
    buffers run past one 64-buffer metadata window."""
    rng = np.random.default_rng(3)
    lens = rng.integers(64, 200, 60_000)
    offs, host = _packed(port, lens, 0, 0x33, lead=5)
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, 3, mask_too=False)


def test_region_workspace_and_host(dev, C, port):
    """Caller workspace (exact size; ENOSPC when one byte short) and the host
    region entry point, which takes the region path for sorted batches."""
    rng = np.random.default_rng(9)
    lens = rng.integers(1, 9000, 700)
    offs, host = _packed(port, lens, 5, 0x99)
    buf = torch.from_numpy(host).to(dev)
    wsb = C.region_workspace_bytes(len(host), len(offs))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64))
    assert np.array_equal(_region(C, dev, buf, offs, lens, ws=ws), want)
    from nvlevelz_amd import _lib
    rc = _lib.lib.nvl_crc32c_region_dev(buf.data_ptr(), len(host), _t64(offs, dev).data_ptr(),
                                        _t64(lens, dev).data_ptr(), None, 0, ws.data_ptr(), len(offs), 0,
                                        ws.data_ptr(), wsb - 1, None)
    assert rc == -5
    import ctypes
    out = np.zeros(len(offs), dtype=np.uint32)
    o64, l64 = offs.astype(np.uint64), lens.astype(np.uint64)
    rc = _lib.lib.nvl_crc32c_batch_region_host(host.ctypes.data, len(host), o64.ctypes.data, l64.ctypes.data,
                                               None, 0, out.ctypes.data, len(offs), 0)
    assert rc == 0 and np.array_equal(out, want)
    del ctypes
