"""GPU parity: the HIP engine through the C ABI vs the oracle and the
reference-generated golden vectors.  Bit-exact everywhere (integer work).

Sizes: full BASELINE configs 2, 3 and 4 run here (config 4 checked through
its golden digest -- a checksum of checksums -- since its 10 GiB input is not
copied back to the host); everything else compares every CRC with the oracle.
"""
import threading

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


def _dev_bytes(data: bytes, dev, pad: int = 64):
    a = np.zeros(len(data) + pad, dtype=np.uint8)
    a[:len(data)] = np.frombuffer(data, dtype=np.uint8)
    return torch.from_numpy(a).to(dev)


def _varlen(C, dev, buf, offs, lens, init=0, mask=False):
    o = torch.from_numpy(np.asarray(offs, dtype=np.int64)).to(dev)
    m = torch.from_numpy(np.asarray(lens, dtype=np.int64)).to(dev)
    if not isinstance(init, int):
        init = torch.from_numpy(np.asarray(init, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    return _u32(C.extend_batch(buf, o, m, init, mask=mask))


def test_probe_and_gpu_backend(dev, C):
    assert C.gpu_accelerated()


def test_kat_vectors(dev, C):
    g = load_golden("kat")
    blobs = [bytes.fromhex(v["hex"]) for v in g["value"]]
    offs, pos, data = [], 0, b""
    for b in blobs:
        pos += 7  # deliberately unaligned starts
        data += b"\x5a" * 7 + b
        offs.append(pos)
        pos += len(b)
    got = _varlen(C, dev, _dev_bytes(data, dev), offs, [len(b) for b in blobs])
    assert [int(x) for x in got] == [v["crc"] for v in g["value"]]
    ext = g["extend"]
    data = b"".join(bytes.fromhex(e["hex"]) for e in ext)
    offs = np.cumsum([0] + [len(bytes.fromhex(e["hex"])) for e in ext])[:-1]
    got = _varlen(C, dev, _dev_bytes(data, dev), offs, [len(bytes.fromhex(e["hex"])) for e in ext],
                  init=[e["init"] for e in ext])
    assert [int(x) for x in got] == [e["crc"] for e in ext]


def test_sweep_golden(dev, C, port):
    g = load_golden("sweep")
    host = port.fill(g["seed"], 0, g["stream_bytes"])
    buf = torch.from_numpy(host).to(dev)  # torch allocations are >= 256-B aligned
    assert buf.data_ptr() % 256 == 0
    offs, lens, want = [], [], []
    for oi, o in enumerate(g["offsets"]):
        for li, n in enumerate(g["lengths"]):
            offs.append(o)
            lens.append(n)
            want.append(g["crc"][oi][li])
    got = _varlen(C, dev, buf, offs, lens)
    assert np.array_equal(got, np.array(want, dtype=np.uint32))
    ext = g["extend"]
    got = _varlen(C, dev, buf, [e[0] for e in ext], [e[1] for e in ext], init=[e[2] for e in ext])
    assert [int(x) for x in got] == [e[3] for e in ext]


def test_fill_matches_oracle(dev, C, port):
    buf = torch.empty(64 * 4096, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, 64, 4096, 0x5EED0001, first_block=3, block_step=5)
    h = buf.cpu().numpy()
    for k in (0, 1, 63):
        assert np.array_equal(h[k * 4096:(k + 1) * 4096], port.fill(0x5EED0001, (3 + 5 * k) * 4096, 4096))


def test_config2_full(dev, C, port):
    """BASELINE config 2: 10^5 x 4 KiB, device-resident, fast path."""
    g = load_golden("configs")["cfg2"]
    n, L = g["n"], g["len"]
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, n, L, g["seed"])
    got = _u32(C.extend_fixed(buf, L, L, n))
    assert [int(x) for x in got[:8]] == g["crc_first"]
    assert int(got[-1]) == g["crc_last"]
    assert port.digest(got) == g["digest"]
    want = port.fixed(buf.cpu().numpy(), L, L, n)
    assert np.array_equal(got, want)
    # Mask flag = the on-disk trailer value
    gotm = _u32(C.extend_fixed(buf, L, L, n, mask=True))
    assert all(int(gotm[i]) == port.mask(int(want[i])) for i in range(0, n, 97))


def test_config3_full(dev, C, port):
    """BASELINE config 3: 1 GiB packed, 512 B - 64 KiB, unaligned starts."""
    g = load_golden("configs")["cfg3"]
    lens = port.cfg3_lengths(g["len_seed"], g["total"])
    assert lens.size == g["n"] and lens[0] == g["len_first"] and lens[-1] == g["len_last"]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    total = g["total"]
    buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, (total + 64) // 8, 8, g["seed"])
    got = _varlen(C, dev, buf, offs, lens.astype(np.int64))
    assert [int(x) for x in got[:8]] == g["crc_first"]
    assert int(got[-1]) == g["crc_last"]
    assert port.digest(got) == g["digest"]
    want = port.varlen(buf.cpu().numpy(), offs.astype(np.uint64), lens)
    assert np.array_equal(got, want)
    # The same buffers in a random order: not region-shaped, so
    # nvl_crc32c_batch_dev's route runs the batch kernels (head + body) at
    # full config-3 size -- the packed order above takes the region path.
    perm = np.random.default_rng(3).permutation(lens.size)
    got_p = _varlen(C, dev, buf, offs[perm], lens.astype(np.int64)[perm])
    assert np.array_equal(got_p, want[perm])


def test_config4_full(dev, C, port):
    """BASELINE config 4: 5000 x 2 MiB (10 GiB) -- multi-chunk, multi-wave buffers."""
    g = load_golden("configs")["cfg4"]
    n, L = g["n"], g["len"]
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, n, L, g["seed"])
    got = _u32(C.extend_fixed(buf, L, L, n))
    assert [int(x) for x in got[:8]] == g["crc_first"]
    assert int(got[-1]) == g["crc_last"]
    assert port.digest(got) == g["digest"]
    # same buffers through the variable-length path
    offs = np.arange(n, dtype=np.int64) * L
    got2 = _varlen(C, dev, buf, offs, np.full(n, L, dtype=np.int64))
    assert np.array_equal(got, got2)
    del buf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("length", [0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 100, 1000, 4095, 4096, 4097,
                                    8191, 8192, 8193, 12288, 65536, 100003, 2 * 4096 * 64 + 5])
@pytest.mark.parametrize("base_off", [0, 3, 16])
def test_fixed_general(dev, C, port, length, base_off):
    rng = np.random.default_rng(length * 31 + base_off)
    stride = length + int(rng.integers(0, 40))
    if base_off == 16:
        stride = ((length + 15) // 16) * 16  # aligned, maybe not 4096-multiple
    n = max(1, min(300, (6 << 20) // max(stride, 1)))
    total = base_off + (n - 1) * stride + length + 64
    host = port.fill(int(rng.integers(1, 1 << 40)), 0, total)
    buf = torch.from_numpy(host).to(dev)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    init_t = torch.from_numpy(inits.view(np.int32)).to(dev)
    got = _u32(C.extend_fixed(buf, stride, length, n, init_t, base_offset=base_off))
    want = port.fixed(host[base_off:], stride, length, n, inits)
    assert np.array_equal(got, want)
    got = _u32(C.extend_fixed(buf, stride, length, n, 0xDEADBEEF, base_offset=base_off, mask=True))
    want = np.array([port.mask(port.extend(0xDEADBEEF, host[base_off + i * stride:base_off + i * stride + length]))
                     for i in range(n)], dtype=np.uint32)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n", [1, 2, 3, 7, 37, 129])
def test_fixed_multichunk_wave_straddles(dev, C, port, n):
    """Buffers of many chunks cut across wave ranges at odd points (fix-up path)."""
    L = 4096 * 67 + 4096  # 68 chunks each
    host = port.fill(0xABC + n, 0, n * L)
    buf = torch.from_numpy(host).to(dev)
    got = _u32(C.extend_fixed(buf, L, L, n, 0x1234))
    assert np.array_equal(got, port.fixed(host, L, L, n, np.full(n, 0x1234, dtype=np.uint32)))


def test_varlen_random_edges(dev, C, port):
    rng = np.random.default_rng(77)
    n = 3000
    choices = np.array([0, 1, 2, 3, 4, 5, 7, 8, 31, 63, 64, 65, 511, 512, 513, 4095, 4096, 4097, 8192,
                        12289, 65536, 300001])
    lens = np.where(rng.random(n) < 0.5, rng.choice(choices, n), rng.integers(0, 20000, n)).astype(np.int64)
    gaps = rng.integers(0, 33, n)
    offs = (np.cumsum(lens + gaps) - lens).astype(np.int64)
    total = int(offs[-1] + lens[-1]) + 64
    host = port.fill(0x777, 0, total)
    buf = torch.from_numpy(host).to(dev)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _varlen(C, dev, buf, offs, lens, init=inits)
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), inits)
    assert np.array_equal(got, want)
    # shuffled order and overlapping buffers are legal too
    perm = rng.permutation(n)
    got = _varlen(C, dev, buf, offs[perm], lens[perm], init=inits[perm], mask=True)
    assert np.array_equal(got, np.array([port.mask(int(x)) for x in want[perm]], dtype=np.uint32))


def test_varlen_long_heads_page_edges(dev, C, port):
    """Long heads (1025..4095 B), which the head kernel runs as whole chunks
    with row loads reaching up to 12 bytes below the buffer's 16-B granule,
    at starts around 4 KiB page boundaries of the absolute address: a buffer
    starting in a page's first granule takes the lane-group path instead
    (tests/kernel_model.py long_head).  1..3 chunks, random inits."""
    rng = np.random.default_rng(4096)
    total = 260 * 4096
    host = port.fill(0xF00D, 0, total)
    buf = torch.from_numpy(host).to(dev)
    base = buf.data_ptr()
    page_offs = [0, 1, 3, 4, 15, 16, 17, 28, 31, 32, 4079, 4080, 4095]
    offs, lens = [], []
    for k in range(400):
        po = page_offs[k % len(page_offs)]
        hl = int(rng.choice([1025, 1026, 1100, 2048, 3000, 4000, 4080, 4081, 4094, 4095]))
        J = int(rng.choice([1, 1, 2, 3]))
        page = 1 + (k * 37) % 240
        offs.append(page * 4096 + (po - base) % 4096)
        lens.append(hl + 4096 * (J - 1))
    offs = np.array(offs, dtype=np.int64)
    lens = np.array(lens, dtype=np.int64)
    assert int((offs + lens).max()) < total
    inits = rng.integers(0, 2**32, size=len(offs), dtype=np.uint64).astype(np.uint32)
    got = _varlen(C, dev, buf, offs, lens, init=inits)
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), inits)
    assert np.array_equal(got, want)
    # the same heads as a fixed-stride batch (the head kernel with FixedGeom)
    for hl in (1025, 3000, 4095):
        for po in (0, 16, 4080):
            off = 4096 + (po - base) % 4096
            n = 50
            got = _u32(C.extend_fixed(buf, hl + 7, hl, n, 0x5A5A5A5A, base_offset=off))
            ref = port.fixed(host[off:], hl + 7, hl, n, np.full(n, 0x5A5A5A5A, dtype=np.uint32))
            assert np.array_equal(got, ref), (hl, po)


def test_varlen_many_tiny(dev, C, port):
    rng = np.random.default_rng(3)
    n = 200_000
    lens = rng.integers(0, 9, n).astype(np.int64)
    offs = rng.integers(0, 1 << 20, n).astype(np.int64)
    host = port.fill(0x99, 0, (1 << 20) + 64)
    buf = torch.from_numpy(host).to(dev)
    got = _varlen(C, dev, buf, offs, lens, init=7)
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), np.full(n, 7, dtype=np.uint32))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n", [1, 2, 1023, 1025, 32767, 32768, 32769, 150_000])
def test_varlen_plan_paths(dev, C, port, n):
    """Both variable-length plans -- one-workgroup (n <= 32768) and counts ->
    device scan -> unit map (larger n) -- around the switch-over point."""
    rng = np.random.default_rng(n)
    lens = np.where(rng.random(n) < 0.9, rng.integers(0, 600, n), rng.integers(0, 30000, n)).astype(np.int64)
    offs = (np.cumsum(lens + 1) - lens).astype(np.int64)
    total = int(offs[-1] + lens[-1]) + 64
    host = port.fill(0x51A + n, 0, total)
    buf = torch.from_numpy(host).to(dev)
    got = _varlen(C, dev, buf, offs, lens, init=0x89ABCDEF)
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), np.full(n, 0x89ABCDEF, dtype=np.uint32))
    assert np.array_equal(got, want)


def test_varlen_lpt_fallback(dev, C, port):
    """Scheduler C hands a workgroup's buffers out most-chunks-first when the
    range holds multi-chunk buffers and at most kPermMax (1792) buffers;
    700k mostly tiny buffers with 2 % of 9000 B ones put ~2700 buffers in
    every workgroup's range: the natural-order fallback."""
    rng = np.random.default_rng(1792)
    n = 700_000
    lens = np.where(rng.random(n) < 0.98, rng.integers(0, 65, n), 9000).astype(np.int64)
    offs = (np.cumsum(lens + 3) - lens).astype(np.int64)
    total = int(offs[-1] + lens[-1]) + 64
    host = port.fill(0x1792, 0, total)
    buf = torch.from_numpy(host).to(dev)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _varlen(C, dev, buf, offs, lens, init=inits)
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), inits)
    assert np.array_equal(got, want)


def test_empty_batches(dev, C):
    buf = torch.zeros(16, dtype=torch.uint8, device=dev)
    assert C.extend_fixed(buf, 0, 0, 0).numel() == 0
    e = torch.empty(0, dtype=torch.int64, device=dev)
    assert C.extend_batch(buf, e, e).numel() == 0
    got = _u32(C.extend_fixed(buf, 0, 0, 5, 0x1234567))
    assert list(got) == [0x1234567] * 5  # Extend(c, "", 0) == c


def test_single_bit_errors_detected_full_size(dev, C):
    """Size-independent property at config-2 size: every 1-bit corruption changes the CRC."""
    n, L = 100_000, 4096
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, n, L, 0x5EED0001)
    before = C.extend_fixed(buf, L, L, n).clone()
    rng = np.random.default_rng(11)
    pos = torch.from_numpy(rng.integers(0, L, n) + np.arange(n) * L).to(dev)
    bit = torch.from_numpy((1 << rng.integers(0, 8, n)).astype(np.uint8)).to(dev)
    buf[pos] ^= bit
    after = C.extend_fixed(buf, L, L, n)
    assert bool((before != after).all())
    buf[pos] ^= bit
    assert torch.equal(before, C.extend_fixed(buf, L, L, n))


def test_extend_composition_full_size(dev, C):
    """Extend(Value(A), B) == Value(A||B) (util/crc32c_test.cc:54-57) for 10^5 splits."""
    n, L = 100_000, 4096
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, n, L, 0x5EED0001)
    whole = C.extend_fixed(buf, L, L, n)
    first = C.extend_fixed(buf, L, 1000, n)
    second = C.extend_fixed(buf, L, L - 1000, n, first, base_offset=1000)
    assert torch.equal(whole, second)


def test_host_entry_points(dev, C, port):
    rng = np.random.default_rng(8)
    blobs = [port.fill(i, 0, int(rng.integers(0, 70000))).tobytes() for i in range(50)]
    inits = [int(x) for x in rng.integers(0, 2**32, 50)]
    got = C.extend_batch_host(blobs, inits, mask=True)
    assert [int(x) for x in got] == [port.mask(port.extend(i, b)) for i, b in zip(inits, blobs)]
    host = port.fill(5, 0, 3000 * 4096)
    got = C.extend_fixed_host(host, 4096, 4096, 3000)
    assert np.array_equal(got, port.fixed(host, 4096, 4096, 3000))


def test_region_host_sliced_staging(dev, C, port):
    """nvl_crc32c_batch_region_host over a ~75 MB window that starts at a
    non-zero offset and is not a multiple of the 8 MiB staging slice (the
    4-thread sliced copy + per-slice H2D path), every CRC against the oracle."""
    import ctypes
    from nvlevelz_amd import _lib
    region = port.fill(0x77, 0, 80_000_000)
    rng = np.random.default_rng(21)
    n = 3000
    lo, hi = 1_234_567, 76_543_211
    lens = rng.integers(0, 70_000, size=n).astype(np.uint64)
    offs = (lo + (rng.random(n) * (hi - lo - lens)).astype(np.uint64)).astype(np.uint64)
    offs[0], lens[0] = lo, 5
    offs[1], lens[1] = hi - 17, 17
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    rc = _lib.lib.nvl_crc32c_batch_region_host(region.ctypes.data, region.nbytes, offs.ctypes.data, lens.ctypes.data,
                                               inits.ctypes.data, 0, out.ctypes.data, n, 0)
    assert rc == 0, rc
    want = [port.extend(int(i), region[int(o):int(o) + int(m)].tobytes()) for i, o, m in zip(inits, offs, lens)]
    assert [int(x) for x in out] == want


def test_fixed_host_pipe_reuse(dev, C, port):
    """nvl_crc32c_fixed_host keeps its slabs per thread: calls of growing and
    shrinking size (slab regrow, then reuse) all match the oracle."""
    for n, L, seed in [(3000, 4096, 1), (40000, 1024, 2), (700, 2 * 4096 + 3, 3), (3000, 4096, 4)]:
        host = port.fill(seed, 0, n * L)
        got = C.extend_fixed_host(host, L, L, n)
        assert np.array_equal(got, port.fixed(host, L, L, n)), (n, L)


def test_workspace_contract(dev, C):
    from nvlevelz_amd._lib import Crc32cError, ENOSPC
    n, L = 10, 3 * 4096
    buf = torch.zeros(n * L, dtype=torch.uint8, device=dev)
    need = C.fixed_workspace_bytes(L, L, n)
    assert need > 0
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    a = C.extend_fixed(buf, L, L, n, workspace=ws)
    with pytest.raises(Crc32cError) as ei:
        C.extend_fixed(buf, L, L, n, workspace=ws[:need // 2])
    assert ei.value.status == ENOSPC
    assert torch.equal(a, C.extend_fixed(buf, L, L, n))


def test_concurrent_threads_and_streams(dev, C, port):
    host = port.fill(0x31, 0, 4000 * 4096)
    buf = torch.from_numpy(host).to(dev)
    want = port.fixed(host, 4096, 4096, 4000)
    errs = []

    def worker(k):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(5):
                    o = torch.from_numpy((np.arange(4000) * 4096).astype(np.int64)).to(dev)
                    m = torch.full((4000,), 4096, dtype=torch.int64, device=dev)
                    r = C.extend_batch(buf, o, m)
                    s.synchronize()
                    if not np.array_equal(_u32(r), want):
                        errs.append(k)
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs


@pytest.mark.parametrize("J,n,gap", [(2, 300, 0), (3, 100, 4096), (64, 9, 16), (65, 5, 0), (512, 7, 0),
                                     (1000, 3, 32), (127, 2, 4096 * 3)])
def test_fixed_chunk_parallel(dev, C, port, J, n, gap):
    """Aligned multi-chunk buffers (crc32c_chunks_kernel + crc32c_fold_kernel):
    J below, at and above one lane run per lane (R = ceil(J/64)), powers of
    two and not, gaps between buffers, per-buffer inits and Mask."""
    L = 4096 * J
    stride = L + gap
    host = port.fill(0xC4 + J, 0, (n - 1) * stride + L)
    buf = torch.from_numpy(host).to(dev)
    rng = np.random.default_rng(J)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _u32(C.extend_fixed(buf, stride, L, n, torch.from_numpy(inits.view(np.int32)).to(dev)))
    want = port.fixed(host, stride, L, n, inits)
    assert np.array_equal(got, want)
    got = _u32(C.extend_fixed(buf, stride, L, n, 0x0BADF00D, mask=True))
    want = port.fixed(host, stride, L, n, np.full(n, 0x0BADF00D, dtype=np.uint32))
    assert np.array_equal(got, np.array([port.mask(int(x)) for x in want], dtype=np.uint32))


def _page_head_start(base_off, stride, n):
    """Some start base_off + k stride (k < n), offsets from a page start, in
    a page's first 16 bytes."""
    return any(((base_off + k * stride) & 4095) < 16 for k in range(n))


@pytest.mark.parametrize("length", [1025, 1500, 2049, 3500, 4095])
@pytest.mark.parametrize("layout", ["clear", "page_heads"])
def test_fixed_masked_pairs(dev, C, port, length, layout):
    """Fixed-stride batches of one 1025..4095-byte chunk per buffer run as
    masked scheduler-A passes (crc32c_fixed_kernel<kGeneral>, kMasked):
    layouts with no start in a page's first granule, and layouts with such
    starts (page_head_words moves the straddling slot's words); per-buffer
    inits and Mask, odd strides and bases."""
    if layout == "clear":
        base_off, stride = 48, (length + 31) // 32 * 32 + 4096 * ((length // 2048) % 2)
        if stride % 4096 == 0:
            stride += 32
    else:
        base_off, stride = 5, length + 3
    n = 20000
    assert _page_head_start(base_off, stride, n) == (layout == "page_heads")
    rng = np.random.default_rng(length * 7 + len(layout))
    total = 4096 + base_off + (n - 1) * stride + length + 64
    host = port.fill(int(rng.integers(1, 1 << 40)), 0, total)
    buf = torch.from_numpy(host).to(dev)
    base_off += -buf.data_ptr() % 4096  # offsets relative to a page start
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _u32(C.extend_fixed(buf, stride, length, n, torch.from_numpy(inits.view(np.int32)).to(dev),
                              base_offset=base_off))
    want = port.fixed(host[base_off:], stride, length, n, inits)
    assert np.array_equal(got, want)
    got = _u32(C.extend_fixed(buf, stride, length, n, 0x2468ACE1, base_offset=base_off, mask=True))
    want = port.fixed(host[base_off:], stride, length, n, np.full(n, 0x2468ACE1, dtype=np.uint32))
    assert np.array_equal(got, np.array([port.mask(int(x)) for x in want], dtype=np.uint32))


@pytest.mark.parametrize("n,maxlen", [(1, 8192), (5000, 8192), (5000, 8193), (1_200_000, 300)])
def test_region_host_short_batches(dev, C, port, n, maxlen):
    """nvl_crc32c_batch_region_host knows the lengths on the host: when every
    length is <= 8192 (two chunks) and the tiles are small enough for the head
    kernel's short mode, the fused body kernel is not launched at all
    (var_heads_only); 8193 and 1.2M buffers (tiles past one sub-range) keep
    both launches.  Lengths 0..3, 4096..4099 and maxlen itself, starts in a
    page's first granule included."""
    from nvlevelz_amd import _lib
    rng = np.random.default_rng(n + maxlen)
    lens = rng.integers(0, maxlen + 1, size=n).astype(np.uint64)
    special = np.array([0, 1, 2, 3, 4, 4095, 4096, 4097, 4098, 4099, maxlen], dtype=np.uint64)
    special = special[special <= maxlen]
    k = min(n, special.size)
    lens[:k] = special[:k]
    lens[-1] = maxlen
    gaps = rng.integers(0, 20, size=n).astype(np.uint64)
    offs = np.zeros(n, dtype=np.uint64)
    pos = 4096 * 3  # buffer 0 at a page start
    for i in range(n):
        offs[i] = pos
        pos += int(lens[i] + gaps[i])
    region = port.fill(0x5A + n, 0, pos + 64)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    rc = _lib.lib.nvl_crc32c_batch_region_host(region.ctypes.data, region.nbytes, offs.ctypes.data, lens.ctypes.data,
                                               inits.ctypes.data, 0, out.ctypes.data, n, 1)
    assert rc == 0, rc
    want = port.varlen(region, offs, lens, inits)
    assert np.array_equal(out, np.array([port.mask(int(x)) for x in want], dtype=np.uint32))
    if n <= 5000:  # nvl_crc32c_batch_host: the same buffers packed by the library, 16-B aligned starts
        blobs = [region[int(o):int(o) + int(m)].tobytes() for o, m in zip(offs, lens)]
        got = C.extend_batch_host(blobs, [int(x) for x in inits])
        assert np.array_equal(np.asarray(got, dtype=np.uint32), want)


@pytest.mark.parametrize("length,stride,n", [(1025, 1, 5000), (3000, 7, 3000), (4095, 1000, 2000), (2049, 4096, 3),
                                             (3500, 3500, 1), (1100, 16, 2)])
def test_fixed_masked_pairs_overlapping(dev, C, port, length, stride, n):
    """kMasked scheduler-A passes over fixed batches whose buffers overlap
    (stride < len, down to 1 byte: every start alignment and, with a page-
    aligned base, starts in pages' first granules), and tiny n."""
    rng = np.random.default_rng(length * 131 + stride)
    total = 4096 + (n - 1) * stride + length + 64
    host = port.fill(int(rng.integers(1, 1 << 40)), 0, total)
    buf = torch.from_numpy(host).to(dev)
    base_off = -buf.data_ptr() % 4096  # the first buffer at a page start
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _u32(C.extend_fixed(buf, stride, length, n, torch.from_numpy(inits.view(np.int32)).to(dev),
                              base_offset=base_off))
    want = port.fixed(host[base_off:], stride, length, n, inits)
    assert np.array_equal(got, want)


def test_read_probe_reads_every_granule(dev):
    """nvl_crc32c_read_probe (bench.py's measured read ceiling) XORs every
    16-byte granule a thread reads (granules t, t + S, t + 2S, ..., S = 256 x
    1024 threads) and writes its sink only when that XOR is 0x12345678.  The
    pattern split over two granules S apart -- the last one and the one a
    stride before it -- reaches the sink only if that thread read both, in
    the four-load main loop, the tail loop, or across them."""
    from nvlevelz_amd import _lib
    lib = _lib.lib
    st = torch.cuda.current_stream().cuda_stream
    S = 256 * 1024
    for n16 in (1, 4 * S + 5, 8 * S, 9 * S - 1):
        buf = torch.zeros(n16 * 4, dtype=torch.int32, device=dev)
        if n16 == 1:
            buf[0] = 0x12345678
        else:
            buf[4 * (n16 - 1)] = 0x12340000
            buf[4 * (n16 - 1 - S) + 3] = 0x5678
        sink = torch.zeros(1, dtype=torch.int32, device=dev)
        assert lib.nvl_crc32c_read_probe(buf.data_ptr(), n16 * 16, sink.data_ptr(), st) == 0
        torch.cuda.synchronize()
        assert int(sink.item()) == 0x12345678, n16
        buf[4 * (n16 - 1) + 1] = 1  # now no thread's XOR is the pattern
        sink.zero_()
        assert lib.nvl_crc32c_read_probe(buf.data_ptr(), n16 * 16, sink.data_ptr(), st) == 0
        torch.cuda.synchronize()
        assert int(sink.item()) == 0, n16
