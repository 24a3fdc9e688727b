"""GPU parity at sizes the other suites do not reach: single buffers of
gigabytes (a buffer whose chunks span hundreds of workgroups' ranges, so the
edge records of workgroups wholly inside one buffer are folded), lengths past
2^32 bytes (64-bit offsets and lengths end to end), and fixed-stride batches
of such buffers through the misaligned general path (head kernel + scheduler
B + fix-up).  Every CRC is compared bit for bit with the oracle
(oracle/crc32c_oracle.c, pinned to the reference's util/crc32c.cc)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

GiB = 1 << 30


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


@pytest.fixture(scope="module")
def port():
    import oracle
    return oracle.port()


def _u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def test_varlen_giant_buffers(dev, C, port):
    """Variable-length batch mixing gigabyte buffers with tiny ones: the
    long-buffer plan (scheduler B over the chunk space, per-workgroup edge
    records, the last workgroup's fold) with per-buffer inits and Mask."""
    lens = np.array([7, GiB + 123, 4097, 700 * (1 << 20) + 1, 3, 65536, 2 * GiB - 5, 1, 4096, 0],
                    dtype=np.int64)
    gaps = np.array([1, 3, 0, 5, 2, 7, 1, 0, 3, 1], dtype=np.int64)
    offs = np.zeros_like(lens)
    pos = 13
    for k in range(lens.size):
        offs[k] = pos
        pos += int(lens[k] + gaps[k])
    host = port.fill(0x61A47, 0, pos + 64)
    buf = torch.from_numpy(host).to(dev)
    rng = np.random.default_rng(0x61A47)
    inits = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64).astype(np.uint32)
    o = torch.from_numpy(offs).to(dev)
    m = torch.from_numpy(lens).to(dev)
    got = _u32(C.extend_batch(buf, o, m, torch.from_numpy(inits.view(np.int32)).to(dev)))
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), inits)
    assert np.array_equal(got, want)
    got = _u32(C.extend_batch(buf, o, m, 0x13579BDF, mask=True))
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64),
                       np.full(lens.size, 0x13579BDF, dtype=np.uint32))
    assert np.array_equal(got, np.array([port.mask(int(x)) for x in want], dtype=np.uint32))


def test_length_past_4gib(dev, C, port):
    """One buffer of 4 GiB + 5 bytes from an odd start, as a one-buffer
    variable batch and as a one-buffer fixed batch: 64-bit lengths and
    offsets through the plan, the chunk positions and the fix-up."""
    L = 4 * GiB + 5
    off = 3
    host = port.fill(0x4C1B, 0, off + L + 64)
    buf = torch.from_numpy(host).to(dev)
    want = port.varlen(host, np.array([off], dtype=np.uint64), np.array([L], dtype=np.uint64),
                       np.array([0xA5A5A5A5], dtype=np.uint32))
    o = torch.tensor([off], dtype=torch.int64, device=dev)
    m = torch.tensor([L], dtype=torch.int64, device=dev)
    got = _u32(C.extend_batch(buf, o, m, 0xA5A5A5A5))
    assert int(got[0]) == int(want[0])
    got = _u32(C.extend_fixed(buf[off:], L, L, 1, 0xA5A5A5A5))
    assert int(got[0]) == int(want[0])


@pytest.mark.parametrize("L,n,stride_gap,base_off", [(GiB + 3, 3, 5, 1), (256 * (1 << 20) + 4097, 5, 0, 7)])
def test_fixed_general_giant(dev, C, port, L, n, stride_gap, base_off):
    """Misaligned fixed-stride batches of very long buffers (head kernel for
    the partial first chunks, scheduler B across workgroups, fix-up)."""
    stride = L + stride_gap
    total = base_off + (n - 1) * stride + L
    host = port.fill(0x9E7 + n, 0, total + 64)
    buf = torch.from_numpy(host).to(dev)
    rng = np.random.default_rng(L)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _u32(C.extend_fixed(buf[base_off:], stride, L, n, torch.from_numpy(inits.view(np.int32)).to(dev)))
    want = port.fixed(host[base_off:], stride, L, n, inits)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("J,n", [(1025, 3), (2049, 2), (5127, 1), (262144, 1), (4096, 2)])
def test_fixed_aligned_long_buffers(dev, C, port, J, n):
    """Aligned fixed-stride batches of buffers longer than the one-level
    chunk fold takes (J > 1024 chunks: the two-level fold over segments of
    1024 chunk raws, first segment clipped), incl. a lone 1 GiB buffer, with
    per-buffer inits and Mask."""
    L = J * 4096
    host = port.fill(0xA1A + J, 0, n * L)
    buf = torch.from_numpy(host).to(dev)
    rng = np.random.default_rng(J)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _u32(C.extend_fixed(buf, L, L, n, torch.from_numpy(inits.view(np.int32)).to(dev)))
    want = port.fixed(host, L, L, n, inits)
    assert np.array_equal(got, want)
    gotm = _u32(C.extend_fixed(buf, L, L, n, mask=True))
    want0 = port.fixed(host, L, L, n)
    assert [int(x) for x in gotm] == [port.mask(int(x)) for x in want0]
