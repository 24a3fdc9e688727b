"""GPU parity of routed calls: nvl_crc32c_batch_dev and
nvl_crc32c_region_dev over device metadata run crc32c_route_plan, then the
region path when the batch is region-shaped (sorted, non-overlapping, every
buffer <= 128 KiB; batch_dev also: gaps <= 1/8 of the bytes + 64 KiB, the
region being the batch's own span) and the head + body kernels otherwise.

Every CRC is compared with the oracle, on both sides of each rule's
boundary: region shapes through batch_dev (offsets from a base and absolute
addresses), the 128 KiB length limit, the gap rule, unsorted / overlapping /
outside-the-region batches through region_dev, zero-length batches, and
alternating routes on one stream with one workspace."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

MAXLEN = 128 << 10


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
    return torch.from_numpy(np.asarray(a, dtype=np.uint64).view(np.int64)).to(dev)


def _inits(n, seed):
    return np.random.default_rng(seed).integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)


def _tinit(inits, dev):
    return torch.from_numpy(inits.view(np.int32)).to(dev)


def _packed(lens, gaps, lead=0):
    lens = np.asarray(lens, dtype=np.int64)
    gaps = np.broadcast_to(np.asarray(gaps, dtype=np.int64), lens.shape)
    offs = (lead + np.cumsum(lens + gaps) - lens - gaps).astype(np.int64)
    return offs


def _both(C, dev, port, host, buf, offs, lens, seed, mask=False):
    """batch_dev and region_dev (region = the whole buffer) against the oracle."""
    inits = _inits(len(offs), seed)
    want = port.varlen(host, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint64), inits)
    if mask:
        want = np.array([port.mask(int(x)) for x in want], dtype=np.uint32)
    o, l, i = _t64(offs, dev), _t64(lens, dev), _tinit(inits, dev)
    got_b = _u32(C.extend_batch(buf, o, l, i, mask=mask))
    got_r = _u32(C.extend_region(buf, o, l, i, mask=mask))
    for name, got in (("batch_dev", got_b), ("region_dev", got_r)):
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (name, bad[:8], np.asarray(offs)[bad[:8]], np.asarray(lens)[bad[:8]])


@pytest.mark.parametrize("shape", ["r", "v", "cfg3", "mixed", "tiny", "one"])
def test_region_shapes_through_both_entries(dev, C, port, shape):
    """Region-shaped batches: the route takes the region path on both entry
    points (the batch's span is its own region on batch_dev)."""
    rng = np.random.default_rng(hash(shape) & 0xFFFF)
    if shape == "r":
        lens = rng.integers(3364, 4110, 30_000)
        offs = _packed(lens, 4, lead=int(rng.integers(0, 4096)))
    elif shape == "v":
        lens = np.full(20_000, 4097)
        offs = _packed(lens, 0, lead=4093)
    elif shape == "cfg3":
        lens = 512 + rng.integers(0, 65025, 3000)
        offs = _packed(lens, 0, lead=0)
    elif shape == "mixed":  # 0..128 KiB, small gaps (region-shaped: gaps << bytes)
        lens = np.where(rng.random(4000) < 0.1, rng.integers(0, 64, 4000), rng.integers(64, MAXLEN + 1, 4000))
        offs = _packed(lens, rng.integers(0, 40, 4000), lead=17)
    elif shape == "tiny":  # every buffer < 64 B (folded whole), still sorted and dense
        lens = rng.integers(1, 64, 5000)
        offs = _packed(lens, 0, lead=3)
    else:
        lens = np.array([MAXLEN])
        offs = np.array([5])
    host = port.fill(0xB0 + len(shape), 0, int(offs[-1] + lens[-1]) + 4096)
    _both(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, 7, mask=shape == "v")


def test_length_limit_boundary(dev, C, port):
    """A buffer of 128 KiB keeps the batch on the region path, one byte more
    sends it to the batch path: both correct, in the same order of calls."""
    for extra in (0, 1, 0):
        lens = np.array([4000, MAXLEN + extra, 4097, 70_000])
        offs = _packed(lens, 3, lead=100)
        host = port.fill(0x128 + extra, 0, int(offs[-1] + lens[-1]) + 64)
        _both(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, extra)


def test_gap_rule_boundary(dev, C, port):
    """batch_dev reads the gaps on the region path: a sparse sorted batch (gaps
    of 1 MiB between 4 KiB buffers) takes the batch path, a dense one the
    region path -- both right; region_dev has no gap rule (its region is the
    caller's)."""
    lens = np.full(200, 4096)
    for gap in (1 << 20, 100, 0):
        offs = _packed(lens, gap, lead=11)
        host = port.fill(0x6A9, 0, int(offs[-1] + lens[-1]) + 64)
        _both(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, gap)


def test_absolute_addresses(dev, C, port):
    """batch_dev with base = NULL: offsets are device addresses (region-shaped
    and not), the plan's span in address space."""
    from nvlevelz_amd import _lib
    rng = np.random.default_rng(4)
    lens = rng.integers(1000, 9000, 3000)
    offs = _packed(lens, 2, lead=9)
    host = port.fill(0xAB5, 0, int(offs[-1] + lens[-1]) + 64)
    buf = torch.from_numpy(host).to(dev)
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64))
    for perm in (np.arange(len(offs)), rng.permutation(len(offs))):
        addr = (buf.data_ptr() + offs[perm]).astype(np.uint64)
        out = torch.empty(len(offs), dtype=torch.int32, device=dev)
        # (the metadata tensors held until the call has run: a temporary's
        # memory goes back to the caching allocator at once)
        ta, tl = _t64(addr, dev), _t64(lens[perm], dev)
        rc = _lib.lib.nvl_crc32c_batch_dev(None, ta.data_ptr(), tl.data_ptr(), None, 0, out.data_ptr(), len(offs), 0,
                                           None, 0, torch.cuda.current_stream(dev).cuda_stream)
        assert rc == 0
        assert np.array_equal(_u32(out), want[perm])


def test_region_dev_non_conforming(dev, C, port):
    """Through region_dev: a permuted 10^4 x 4 KiB batch, overlapping
    buffers, one buffer outside the region, and a batch with one 300 KB
    buffer -- the route sends each to the batch path (never a lane per
    buffer) and each comes out right; the region path right after."""
    rng = np.random.default_rng(8)
    n = 10_000
    host = port.fill(0x9E, 0, n * 4096 + 4096)
    buf = torch.from_numpy(host).to(dev)
    offs = rng.permutation(n).astype(np.int64) * 4096
    lens = np.full(n, 4096)
    _both(C, dev, port, host, buf, offs, lens, 1)
    offs2 = np.sort(rng.integers(0, n * 4096 - 9000, 2000)).astype(np.int64)
    lens2 = rng.integers(1, 9000, 2000)  # sorted starts, overlapping buffers
    _both(C, dev, port, host, buf, offs2, lens2, 2)
    region = buf[:100_000]
    offs3 = np.array([10, 5000, 99_000])
    lens3 = np.array([4000, 90_000, 5000])  # the last one ends past the region (inside the allocation)
    want = port.varlen(host, offs3.astype(np.uint64), lens3.astype(np.uint64))
    assert np.array_equal(_u32(C.extend_region(region, _t64(offs3, dev), _t64(lens3, dev))), want)
    lens4 = np.array([5000, 300_000, 12])
    offs4 = _packed(lens4, 1)
    _both(C, dev, port, host, buf, offs4, lens4, 4)
    lens5 = rng.integers(3364, 4110, 5000)
    _both(C, dev, port, host, buf, _packed(lens5, 4), lens5, 5)


def test_alternating_routes_one_workspace(dev, C, port):
    """Region-shaped and non-region batches alternate on one stream with one
    caller workspace (sized for the larger): the plan is rewritten by every
    call and the event records carry the call's generation and index."""
    rng = np.random.default_rng(12)
    n = 4000
    host = port.fill(0xA17, 0, n * 5000 + 8192)
    buf = torch.from_numpy(host).to(dev)
    lens = rng.integers(3000, 5000, n)
    sorted_offs = _packed(lens, 1)
    perm = rng.permutation(n)
    wsb = max(C.batch_workspace_bytes(n), C.region_workspace_bytes(buf.numel(), n))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    for k in range(6):
        offs = sorted_offs if k % 2 == 0 else sorted_offs[perm]
        ln = lens if k % 2 == 0 else lens[perm]
        want = port.varlen(host, offs.astype(np.uint64), ln.astype(np.uint64))
        f = C.extend_batch if k % 3 else C.extend_region
        got = _u32(f(buf, _t64(offs, dev), _t64(ln, dev), workspace=ws))
        assert np.array_equal(got, want), k


def test_zero_length_and_single(dev, C, port):
    host = port.fill(0x0, 0, 8192)
    buf = torch.from_numpy(host).to(dev)
    for offs, lens in (([0, 0, 5, 5], [0, 0, 0, 0]), ([100], [0]), ([4095], [1]), ([0], [8192])):
        _both(C, dev, port, host, buf, np.array(offs), np.array(lens), 0)


def test_page_rule_boundary(dev, C, port):
    """batch_dev's page rule (crc32c_route_plan `pages`) around its boundary:
    the next buffer starting one page past the previous one's last page or
    inside the page after it (offsets from a tensor whose address is only
    512-B aligned, so the cases fall on both sides of the rule).  Both routes
    right, in mapped memory."""
    for lead, nxt in ((0, 8192), (0, 8191), (4092, 4100), (4092, 4000), (5, 4096 + 4091)):
        lens = np.array([4096 - lead % 4096 if lead else 4096, 9000, 3000])
        offs = np.array([lead, lead + nxt, lead + nxt + 9000 + 2])
        host = port.fill(0x9A6 + nxt, 0, int(offs[-1] + lens[-1]) + 64)
        _both(C, dev, port, host, torch.from_numpy(host).to(dev), offs, lens, nxt)


def test_unmapped_page_between_buffers(dev, C, port):
    """Two device mappings with an unmapped hole between them (HIP virtual
    memory: one address reservation, two physical allocations mapped around a
    hole of one granule) and a sorted batch of 128 KiB buffers on both sides,
    by absolute address: the hole is small against the bytes (the gap rule
    alone would take the region path, which reads every page of the span and
    would fault in the hole); the page rule sends it to the batch path, which
    reads only the buffers.  Skipped where the virtual memory API is missing."""
    import ctypes as ct
    from nvlevelz_amd import _lib  # noqa: F401  (loads the HIP runtime the engine links)
    hip = ct.CDLL("libamdhip64.so.7")

    class Loc(ct.Structure):
        _fields_ = [("type", ct.c_int), ("id", ct.c_int)]

    class Flags(ct.Structure):
        _fields_ = [("compressionType", ct.c_ubyte), ("gpuDirectRDMACapable", ct.c_ubyte), ("usage", ct.c_ushort)]

    class Prop(ct.Structure):
        _fields_ = [("type", ct.c_int), ("requestedHandleType", ct.c_int), ("location", Loc),
                    ("win32HandleMetaData", ct.c_void_p), ("allocFlags", Flags)]

    class Access(ct.Structure):
        _fields_ = [("location", Loc), ("flags", ct.c_int)]

    for f in ("hipMemGetAllocationGranularity", "hipMemAddressReserve", "hipMemCreate", "hipMemMap",
              "hipMemSetAccess", "hipMemUnmap", "hipMemRelease", "hipMemAddressFree", "hipMemcpy"):
        getattr(hip, f).restype = ct.c_int
    torch.cuda.synchronize(dev)
    prop = Prop(1, 0, Loc(1, dev.index or 0), None, Flags(0, 0, 0))
    gran = ct.c_size_t(0)
    if hip.hipMemGetAllocationGranularity(ct.byref(gran), ct.byref(prop), 0) != 0 or gran.value == 0:
        pytest.skip("hipMemGetAllocationGranularity unavailable")
    H = gran.value                                   # the hole: one granule
    D = -(-(24 << 20) // H) * H                      # each mapping
    va = ct.c_void_p(0)
    assert hip.hipMemAddressReserve(ct.byref(va), ct.c_size_t(2 * D + H), ct.c_size_t(0), None, ct.c_ulonglong(0)) == 0
    handles, mapped = [], []
    try:
        for k in range(2):
            h = ct.c_void_p(0)
            if hip.hipMemCreate(ct.byref(h), ct.c_size_t(D), ct.byref(prop), ct.c_ulonglong(0)) != 0:
                pytest.skip("hipMemCreate unavailable")
            handles.append(h)
            at = va.value + k * (D + H)
            assert hip.hipMemMap(ct.c_void_p(at), ct.c_size_t(D), ct.c_size_t(0), h, ct.c_ulonglong(0)) == 0
            mapped.append(at)
            acc = Access(Loc(1, dev.index or 0), 3)
            assert hip.hipMemSetAccess(ct.c_void_p(at), ct.c_size_t(D), ct.byref(acc), ct.c_size_t(1)) == 0
        img = port.fill(0x401E, 0, 2 * D + H)
        for at in mapped:
            rel = at - va.value
            assert hip.hipMemcpy(ct.c_void_p(at), img[rel:rel + D].ctypes.data_as(ct.c_void_p), ct.c_size_t(D), 1) == 0
        L = 128 << 10
        k1 = D // L
        rel = np.concatenate([np.arange(k1) * L, D + H + np.arange(k1) * L]).astype(np.int64)
        lens = np.full(rel.size, L)
        assert (rel[k1] - (rel[k1 - 1] + L)) <= lens.sum() // 8 + 65536  # the gap rule would pass
        want = port.varlen(img, rel.astype(np.uint64), lens.astype(np.uint64))
        ta, tl = _t64((va.value + rel).astype(np.uint64), dev), _t64(lens, dev)
        out = torch.empty(rel.size, dtype=torch.int32, device=dev)
        rc = _lib.lib.nvl_crc32c_batch_dev(None, ta.data_ptr(), tl.data_ptr(), None, 0, out.data_ptr(), rel.size, 0,
                                           None, 0, torch.cuda.current_stream(dev).cuda_stream)
        assert rc == 0
        torch.cuda.synchronize(dev)
        assert np.array_equal(_u32(out), want)
    finally:
        torch.cuda.synchronize(dev)
        for at in mapped:
            hip.hipMemUnmap(ct.c_void_p(at), ct.c_size_t(D))
        for h in handles:
            hip.hipMemRelease(h)
        hip.hipMemAddressFree(va, ct.c_size_t(2 * D + H))


def test_partials_past_the_first_64(dev, C, port):
    """10^5 buffers: the plan runs ~98 workgroups, so the verdict reads
    partials beyond lane 63's first (two per lane).  A single pair out of
    order near the end -- in a partial past the 64th -- must send the batch
    to the batch path on both entries; the same batch sorted takes the region
    path.  Every CRC against the oracle."""
    rng = np.random.default_rng(100)
    n = 100_000
    lens = rng.integers(1000, 1200, n)
    offs = _packed(lens, 3, lead=5)
    host = port.fill(0x1E5, 0, int(offs[-1] + lens[-1]) + 64)
    buf = torch.from_numpy(host).to(dev)
    _both(C, dev, port, host, buf, offs, lens, 1)
    swapped = offs.copy()
    j = n - 7
    swapped[[j, j + 1]] = swapped[[j + 1, j]]
    lsw = lens.copy()
    lsw[[j, j + 1]] = lsw[[j + 1, j]]
    _both(C, dev, port, host, buf, swapped, lsw, 2)


def test_million_small_buffers(dev, C, port):
    """10^6 packed buffers of 1..200 bytes through both entries: the plan's
    128 workgroups each loop over ~7800 pairs (several steps), the region
    path folds ~3900 buffers per workgroup; the same batch with one pair
    swapped in the middle takes the batch path.  Every CRC against the
    oracle."""
    rng = np.random.default_rng(10 ** 6)
    n = 1_000_000
    lens = rng.integers(1, 201, n)
    offs = _packed(lens, 0, lead=3)
    host = port.fill(0x1E6, 0, int(offs[-1] + lens[-1]) + 64)
    buf = torch.from_numpy(host).to(dev)
    _both(C, dev, port, host, buf, offs, lens, 3)
    j = n // 2
    offs2, lens2 = offs.copy(), lens.copy()
    offs2[[j, j + 1]] = offs2[[j + 1, j]]
    lens2[[j, j + 1]] = lens2[[j + 1, j]]
    _both(C, dev, port, host, buf, offs2, lens2, 4)


@pytest.mark.parametrize("case", ["shuffled", "shuffled_odd", "strided", "overlapping", "small", "large_shuffled",
                                  "one_not_4096"])
def test_page_route(dev, C, port, case):
    """Batches of exactly-4096-byte buffers that are not region-shaped take
    the page path (scheduler A over the batch's own list, in the body
    kernel): shuffled, from an odd base (realigned passes),
    sorted but far apart (the gap rule fails), overlapping, a handful, 10^5
    shuffled; and with one 4095-byte buffer among them, the head + body
    kernels.  Every CRC against the oracle, with per-buffer init and the mask."""
    rng = np.random.default_rng(abs(hash(case)) & 0xFFFF)
    n = {"small": 5, "large_shuffled": 100_000}.get(case, 3000)
    lead = 3 if case == "shuffled_odd" else 0
    step = {"strided": 12288, "overlapping": 2048}.get(case, 4096)
    offs = lead + step * np.arange(n, dtype=np.int64)
    lens = np.full(n, 4096, dtype=np.int64)
    if case not in ("strided", "overlapping"):
        p = rng.permutation(n)
        offs = offs[p]
    if case == "one_not_4096":
        lens[n // 2] = 4095
    total = int(offs.max() + 4096 + 64)
    host = rng.integers(0, 256, size=total, dtype=np.uint8)
    buf = torch.from_numpy(host).to(dev)
    _both(C, dev, port, host, buf, offs, lens, seed=n + step, mask=(case == "shuffled"))
