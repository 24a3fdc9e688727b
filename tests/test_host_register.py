"""The staging-free host-resident path (nvl_crc32c_host_register, VERDICT r05
"next" item 5): a host range registered once (hipHostRegister, portable |
mapped) is DMA'd from the caller's own pages by nvl_crc32c_batch_region_host
(no staging copy on the CPU), or read in place by the kernels with
NVL_CRC32C_FLAG_HOST_ZERO_COPY.  Anything not inside one registration still
takes the pinned staging (the fallback).

CPU cases (no GPU): argument checks and the no-device behaviour -- a
registration fails loudly, nothing is recorded, zero copy on an unregistered
range is an argument error, and the staged entry is unaffected.
GPU cases: every CRC against the oracle on registered sorted (region kernel)
and unsorted (batch kernels) batches, DMA and zero copy, windows that cross a
registration's end, overlapping registrations refused, the multi-pipe entry
over registered memory, and unregistration."""
import numpy as np
import pytest

from conftest import gpu_present
from nvlevelz_amd import _lib
from nvlevelz_amd import crc32c as C

L = _lib.lib


def _want(port, img, offs, lens, inits=None):
    return port.varlen(img, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint64), inits)


def test_argument_checks():
    a = np.zeros(4096, dtype=np.uint8)
    o = np.zeros(1, dtype=np.uint64)
    m = np.full(1, 100, dtype=np.uint64)
    out = np.zeros(1, dtype=np.uint32)
    assert L.nvl_crc32c_host_register(None, 4096) == _lib.EINVAL
    assert L.nvl_crc32c_host_register(a.ctypes.data, 0) == _lib.EINVAL
    assert L.nvl_crc32c_host_unregister(a.ctypes.data) == _lib.EINVAL  # never registered
    assert L.nvl_crc32c_host_unregister(None) == _lib.EINVAL
    assert L.nvl_crc32c_host_registered(a.ctypes.data, 4096) == 0
    # zero copy needs a registered window; unknown flag bits are refused
    for fl in (_lib.FLAG_HOST_ZERO_COPY, 0x8, 0x2):
        assert L.nvl_crc32c_batch_region_host(a.ctypes.data, a.nbytes, o.ctypes.data, m.ctypes.data, None, 0,
                                              out.ctypes.data, 1, fl) == _lib.EINVAL
    assert out[0] == 0


@pytest.mark.skipif(gpu_present(), reason="checks the no-GPU behaviour")
def test_register_without_a_device_fails_loudly():
    a = np.zeros(1 << 16, dtype=np.uint8)
    rc = L.nvl_crc32c_host_register(a.ctypes.data, a.nbytes)
    assert rc in (_lib.ENODEV, _lib.EHIP)
    assert not C.host_registered(a)  # nothing recorded: later calls take the staging path
    with pytest.raises(C.Crc32cError):
        C.host_register(a)


gpu = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    C.init(0)
    return 0


@gpu
def test_registered_region_dma_and_zero_copy(dev, port):
    rng = np.random.default_rng(6)
    n = 20_000
    lens = rng.integers(3364, 4110, n).astype(np.uint64)  # block | type, 4-byte crc gaps (`r`)
    offs = (np.cumsum(lens + 4) - lens - 4 + 9).astype(np.uint64)
    img = port.fill(0x6E6, 0, int(offs[-1] + lens[-1]) + 100)
    inits = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    want = _want(port, img, offs, lens, inits)
    staged = C.extend_region_host(img, offs, lens, inits)
    assert np.array_equal(staged, want)
    C.host_register(img)
    try:
        assert C.host_registered(img)
        assert L.nvl_crc32c_host_registered(img.ctypes.data + 5, 100) == 1
        assert L.nvl_crc32c_host_registered(img.ctypes.data + img.nbytes - 10, 11) == 0  # runs past the end
        for zc in (False, True, False):
            got = C.extend_region_host(img, offs, lens, inits, zero_copy=zc)
            assert np.array_equal(got, want), zc
            m = C.extend_region_host(img, offs, lens, mask=True, zero_copy=zc)
            assert np.array_equal(m, np.array([port.mask(int(x)) for x in _want(port, img, offs, lens)],
                                              dtype=np.uint32)), zc
        # unsorted / overlapping buffers (the batch kernels) read in place
        perm = rng.permutation(n)[:5000]
        lo = rng.integers(0, 9000, 5000).astype(np.uint64)
        oo = rng.integers(0, img.nbytes - 9000, 5000).astype(np.uint64)
        for zc in (False, True):
            assert np.array_equal(C.extend_region_host(img, offs[perm], lens[perm], zero_copy=zc),
                                  _want(port, img, offs[perm], lens[perm])), zc
            assert np.array_equal(C.extend_region_host(img, oo, lo, zero_copy=zc), _want(port, img, oo, lo)), zc
        # a sub-window of the registration (another view of the same pages)
        sub = img[4097:4097 + 3 * 65536]
        so = np.array([0, 1, 70_000, 131_000], dtype=np.uint64)
        sl = np.array([1, 65_000, 61_000, 65_000], dtype=np.uint64)
        for zc in (False, True):
            assert np.array_equal(C.extend_region_host(sub, so, sl, zero_copy=zc), _want(port, sub, so, sl))
        # overlapping registrations are refused, the first stays
        assert L.nvl_crc32c_host_register(img.ctypes.data + 4096, 4096) == _lib.EINVAL
        assert L.nvl_crc32c_host_register(img.ctypes.data - 4096, 8192) == _lib.EINVAL
        assert C.host_registered(img)
    finally:
        C.host_unregister(img)
    assert not C.host_registered(img)
    with pytest.raises(C.Crc32cError):
        C.extend_region_host(img, offs, lens, zero_copy=True)  # no longer registered
    assert np.array_equal(C.extend_region_host(img, offs, lens, inits), want)  # staging again


@gpu
def test_window_crossing_a_registration_is_staged(dev, port):
    """A batch whose window runs past the registered range takes the pinned
    staging (correct), and zero copy is refused for it."""
    big = port.fill(0x77, 0, 3 << 20)
    head = big[: 1 << 20]
    C.host_register(head)
    try:
        offs = np.array([100, (1 << 20) - 50, 2 << 20], dtype=np.uint64)
        lens = np.array([5000, 100, 4096], dtype=np.uint64)
        assert np.array_equal(C.extend_region_host(big, offs, lens), _want(port, big, offs, lens))
        with pytest.raises(C.Crc32cError):
            C.extend_region_host(big, offs, lens, zero_copy=True)
        inside = offs[:1], lens[:1]
        assert np.array_equal(C.extend_region_host(big, *inside, zero_copy=True), _want(port, big, *inside))
    finally:
        C.host_unregister(head)


@gpu
def test_registered_multi_pipe(dev, port):
    """nvl_crc32c_batch_region_host_multi over registered memory (portable
    registration: every pipe DMAs from the same pages), 2 and 4 pipes into
    the box's one GPU, DMA and zero copy."""
    n, S, Lb = 4000, 4101, 4097
    img = port.fill(0x4444, 0, n * S)
    offs = np.arange(n, dtype=np.uint64) * S
    lens = np.full(n, Lb, dtype=np.uint64)
    want = _want(port, img, offs, lens)
    C.host_register(img)
    try:
        for devs in ([0, 0], [0, 0, 0, 0]):
            for zc in (False, True):
                got = C.extend_region_host(img, offs, lens, devices=devs, min_bytes_per_device=1 << 20, zero_copy=zc)
                assert np.array_equal(got, want), (devs, zc)
    finally:
        C.host_unregister(img)
