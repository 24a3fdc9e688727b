"""The multi-device host entry's cut (nvl_crc32c_multi_plan, CPU) and the
entry itself on the GPU box's one GPU as two and three pipes
(nvl_crc32c_batch_region_host_multi with devices {0, 0} / {0, 0, 0}).

Cut: at most ndev contiguous index ranges covering [0, n), no more than
bytes / min_bytes of them (a small batch stays on one device), each range's
bytes within one buffer of an equal share."""
import numpy as np
import pytest

from nvlevelz_amd import crc32c as C


def _check_plan(lens, ndev, min_bytes):
    lens = np.asarray(lens, dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if lens.size else lens
    first = C.multi_plan(offs, lens, ndev, min_bytes)
    parts = first.size - 1
    total = int(lens.sum())
    mb = min_bytes or (64 << 20)
    assert 1 <= parts <= max(1, min(ndev, total // mb)) or (parts == 1)
    assert first[0] == 0 and first[-1] == lens.size
    assert np.all(np.diff(first.astype(np.int64)) >= 0)
    if parts > 1 and lens.size:
        share = total / parts
        big = int(lens.max())
        for k in range(parts):
            b = int(lens[int(first[k]):int(first[k + 1])].sum())
            assert abs(b - share) <= 2 * big, (k, b, share, big)
    return first


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
def test_plan_equal_blocks(ndev):
    first = _check_plan(np.full(1000, 1 << 20), ndev, 1 << 20)
    assert first.size - 1 == ndev


def test_plan_small_batch_stays_on_one_device():
    assert _check_plan(np.full(10, 4096), 8, 0).size == 2  # 40 KiB < 64 MiB
    assert _check_plan(np.full(100, 1 << 20), 8, 0).size == 2  # 100 MiB: one part of >= 64 MiB
    assert _check_plan(np.full(200, 1 << 20), 8, 0).size == 4  # 200 MiB: three parts


def test_plan_variable_and_degenerate():
    rng = np.random.default_rng(3)
    _check_plan(rng.integers(512, 65536, 32672), 8, 1 << 20)  # config 3's shape
    _check_plan([0] * 50, 4, 1)
    _check_plan([5], 8, 1)
    _check_plan([1 << 30] + [10] * 100, 4, 1 << 20)  # one buffer holds nearly every byte
    first = C.multi_plan(np.zeros(0, np.uint64), np.zeros(0, np.uint64), 4, 1)
    assert first.tolist() == [0, 0]


def test_plan_rejects_bad_arguments():
    from nvlevelz_amd import _lib
    o = np.zeros(4, np.uint64)
    first = np.zeros(3, np.uint64)
    assert _lib.lib.nvl_crc32c_multi_plan(o.ctypes.data, o.ctypes.data, 4, 0, 1, first.ctypes.data) == -1
    assert _lib.lib.nvl_crc32c_multi_plan(None, o.ctypes.data, 4, 2, 1, first.ctypes.data) == -1


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [(0, 0), (0, 0, 0)])
@pytest.mark.parametrize("shape", ["sorted", "shuffled"])
def test_multi_pipes_one_gpu(port, devices, shape):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(len(devices))
    lens = rng.integers(1, 70_000, 1500).astype(np.int64)
    offs = (np.cumsum(lens + 3) - lens - 3).astype(np.int64)
    host = port.fill(0x3170 + len(devices), 0, int(offs[-1] + lens[-1]) + 16)
    if shape == "shuffled":
        p = rng.permutation(lens.size)
        offs, lens = offs[p], lens[p]
    inits = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64).astype(np.uint32)
    want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), inits)
    got = C.extend_region_host(host, offs, lens, inits, devices=devices, min_bytes_per_device=1 << 20)
    assert np.array_equal(got, want)
    got1 = C.extend_region_host(host, offs, lens, inits)
    assert np.array_equal(got1, want)
