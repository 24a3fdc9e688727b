"""GPU parity of the head kernel's short mode (run_heads):
tiles whose buffers all have at most two 4 KiB chunks are finished in the
head kernel itself -- one-chunk buffers as one masked or full pass, two-chunk
buffers as head + body passes in one slot or, with a 1..3-byte head, as the
body pass with the head folded in inline -- and the body kernel exits.

Cases: the SSTable data-block shape (block | type = 3364..4109 B, the `r`
workload), the whole-table-verify shape (4097 B, `v`), full 4096-B and
8192-B buffers, tiny buffers and lane-group heads in the same tiles, a tile
holding two-chunk buffers whose head starts a page's first 16-B granule
(the head in a pre-drain round), a batch whose tiles are mixed (some short, some not: the
body kernel then re-does the short tiles' body chunks from hc), and the
fixed-stride form (nvl_crc32c_fixed_dev with len 4097..4099).  Every CRC is
compared with the oracle, with per-buffer inits and with Mask."""
import numpy as np
import pytest

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


def _check(C, dev, port, host, buf, offs, lens, seed):
    rng = np.random.default_rng(seed)
    n = len(offs)
    o = torch.from_numpy(np.asarray(offs, dtype=np.int64)).to(dev)
    m = torch.from_numpy(np.asarray(lens, dtype=np.int64)).to(dev)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    it = torch.from_numpy(inits.view(np.int32)).to(dev)
    want = port.varlen(host, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint64), inits)
    got = _u32(C.extend_batch(buf, o, m, it))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:10], np.asarray(lens)[bad[:10]], np.asarray(offs)[bad[:10]])
    got = _u32(C.extend_batch(buf, o, m, 0, mask=True))
    want0 = port.varlen(host, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint64))
    assert np.array_equal(got, np.array([port.mask(int(x)) for x in want0], dtype=np.uint32))


def _packed(port, lens, gap, seed, lead=0):
    lens = np.asarray(lens, dtype=np.int64)
    offs = (lead + np.cumsum(lens + gap) - lens - gap).astype(np.int64)
    total = int(offs[-1] + lens[-1]) + 64 if len(lens) else 64
    host = port.fill(seed, 0, total)
    return offs, host


@pytest.mark.parametrize("n", [1, 7, 390, 1024, 3000, 100_000])
def test_sstable_block_shape(dev, C, port, n):
    """block | type of data blocks at block_size 4096 (the `r` workload):
    98 % one masked pass, the rest a body pass with a 1..13-byte head."""
    rng = np.random.default_rng(n)
    lens = rng.integers(3364, 4110, n)
    offs, host = _packed(port, lens, 4, 0x5B + n, lead=int(rng.integers(0, 16)))
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, n)


@pytest.mark.parametrize("gap", [4, 0, 1, 11])
def test_verify_shape_4097(dev, C, port, gap):
    """4096-byte blocks + type byte (`v`): every buffer a body pass with its
    1-byte head inline."""
    n = 20_000
    lens = np.full(n, 4097)
    offs, host = _packed(port, lens, gap, 0x4097 + gap, lead=gap)
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, gap)


def test_short_tile_mixture(dev, C, port):
    """Every kind a short tile holds: tiny (< 4 B), lane-group heads, masked
    passes, full 4096-B passes, 4097..4099 (inline 1..3-byte heads), 4100..8191
    (head + body slots) and 8192 (full head + body)."""
    rng = np.random.default_rng(99)
    choices = np.array([0, 1, 2, 3, 4, 5, 63, 64, 65, 256, 257, 1024, 1025, 1500, 4095, 4096, 4097, 4098, 4099,
                        4100, 4101, 5000, 5120, 8191, 8192])
    n = 20_000
    lens = rng.choice(choices, n)
    sel = rng.random(n) < 0.3
    lens[sel] = rng.integers(0, 8193, int(sel.sum()))
    offs, host = _packed(port, lens, rng.integers(0, 20, n), 0xA11)
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, 5)


def test_page_start_two_chunk_head(dev, C, port):
    """A two-chunk buffer whose 4..4095-byte head starts in a 4 KiB page's
    first 16 bytes cannot be a masked pass: its head runs in a lane-group
    round before the drain and hands its register to the body pass via hc."""
    total = 600 * 4096
    host = port.fill(0xFA11, 0, total)
    buf = torch.from_numpy(host).to(dev)
    base = buf.data_ptr()
    rng = np.random.default_rng(7)
    offs, lens = [], []
    pos = 4096 - base % 4096 + 4096
    for k in range(500):
        L = int(rng.integers(3364, 4110))
        if k % 97 == 13:  # page-start two-chunk buffer with a 4..4095-byte head
            pos = ((base + pos + 4095) // 4096 * 4096 + int(rng.integers(0, 16))) - base
            L = 4096 + int(rng.integers(4, 4096))
        offs.append(pos)
        lens.append(L)
        pos += L + 3
    offs = np.array(offs, dtype=np.int64)
    lens = np.array(lens, dtype=np.int64)
    assert int((offs + lens).max()) < total
    assert any(((base + o) % 4096) < 16 and L > 4100 for o, L in zip(offs, lens))
    _check(C, dev, port, host, buf, offs, lens, 11)


def test_mixed_short_and_long_tiles(dev, C, port):
    """Most tiles short, a few holding a long buffer: the body kernel runs and
    re-does the short tiles' two-chunk bodies from the head kernel's hc."""
    rng = np.random.default_rng(31)
    n = 60_000
    lens = rng.integers(3364, 4110, n)
    lens[rng.random(n) < 0.05] = 4097
    lens[::7919] = 70_000  # J = 18 in a handful of tiles
    offs, host = _packed(port, lens, 4, 0x3131)
    _check(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, 31)


@pytest.mark.parametrize("length", [4097, 4098, 4099])
@pytest.mark.parametrize("extra", [0, 4, 13])
def test_fixed_stride_inline_heads(dev, C, port, length, extra):
    """nvl_crc32c_fixed_dev with len 4097..4099: the fixed head kernel in
    short mode, no body kernel."""
    n = 5000
    stride = length + extra
    for base_off in (0, 1, 6):
        total = base_off + (n - 1) * stride + length + 64
        host = port.fill(length * 7 + extra, 0, total)
        buf = torch.from_numpy(host).to(dev)
        inits = np.random.default_rng(extra).integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        got = _u32(C.extend_fixed(buf, stride, length, n, torch.from_numpy(inits.view(np.int32)).to(dev),
                                  base_offset=base_off))
        assert np.array_equal(got, port.fixed(host[base_off:], stride, length, n, inits)), base_off
        got = _u32(C.extend_fixed(buf, stride, length, n, 0xCAFEF00D, base_offset=base_off, mask=True))
        want = port.fixed(host[base_off:], stride, length, n, np.full(n, 0xCAFEF00D, dtype=np.uint32))
        assert np.array_equal(got, np.array([port.mask(int(x)) for x in want], dtype=np.uint32))
