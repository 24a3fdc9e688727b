"""GPU: BASELINE config 5 at full size on one GPU, the per-device/per-thread
resources of the C ABI, and the measurement entry point.

* Config 5 (BASELINE.json configs[4]): 10^7 x 4 KiB = 41 GB, resident on ONE
  MI355X (288 GB HBM).  Checked against tests/golden/configs.json["cfg5"]
  (oracle restatement pinned block-for-block to the reference build on 10^6
  of the blocks, oracle/gen_golden.py:cfg5): first/last CRCs, the digest of
  all 10^7 CRCs and the ten per-10^6-block sub-digests, plus a random
  sample of blocks re-checksummed by the oracle.
* The host-resident entry points on every visible device from ONE thread,
  and device indices past the count rejected.
* Threads that use the host-resident entry points and exit give their
  device slabs and streams back (no growth over many short-lived threads).
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


def test_config5_full_one_gpu(dev, C, port):
    """10^7 x 4 KiB blocks (41 GB) on one GPU: every CRC via the digest."""
    g = load_golden("configs")["cfg5"]
    n, L = g["n"], g["len"]
    free, _ = torch.cuda.mem_get_info(dev)
    if free < n * L + (4 << 30):
        pytest.skip(f"needs {n * L / 1e9:.0f} GB free HBM, {free / 1e9:.0f} GB free")
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, n, L, g["seed"])
    got = _u32(C.extend_fixed(buf, L, L, n))
    assert [int(x) for x in got[:8]] == g["crc_first"]
    assert int(got[-1]) == g["crc_last"]
    assert port.digest(got) == g["digest"]
    sb = g["sub_digest_blocks"]
    assert [port.digest(got[s:s + sb]) for s in range(0, n, sb)] == g["sub_digests"]
    # a random sample of whole blocks re-checksummed by the oracle on the host
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(n, 512, replace=False))
    sample = buf.view(n, L)[torch.from_numpy(idx).to(dev)].cpu().numpy().reshape(-1)
    assert np.array_equal(got[idx], port.fixed(sample, L, L, idx.size))
    # the same blocks through the round-robin shard layout of 2 and 8 GPUs
    # (rank r holds global blocks r, r+G, ...): shards re-generated in place
    del buf
    torch.cuda.empty_cache()
    for G, r in [(2, 1), (8, 5)]:
        k = (n - r + G - 1) // G
        sh = torch.empty(k * L, dtype=torch.uint8, device=dev)
        C.fill_splitmix(sh, k, L, g["seed"], first_block=r, block_step=G)
        assert np.array_equal(_u32(C.extend_fixed(sh, L, L, k)), got[r::G])
        del sh
        torch.cuda.empty_cache()


@pytest.mark.parametrize("mask,init", [(False, 0), (True, 0x1234ABCD)])
def test_fixed_long_kernel_threshold(dev, C, port, mask, init):
    """Aligned 4 KiB batches of >= 2^18 blocks run crc32c_fixed_long_kernel
    (launch_fixed); one block fewer runs crc32c_fixed_kernel<kAligned>.  Both
    sides of the threshold agree block for block, and a sample with the oracle."""
    L, n = 4096, 1 << 18
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, n, L, 0x5EED0005)
    long_ = _u32(C.extend_fixed(buf, L, L, n, init, mask=mask))
    short = _u32(C.extend_fixed(buf, L, L, n - 1, init, mask=mask))
    assert np.array_equal(long_[:n - 1], short)
    idx = np.array([0, 1, 4095, 4096, n // 2, n - 2, n - 1])
    sample = buf.view(n, L)[torch.from_numpy(idx).to(dev)].cpu().numpy().reshape(-1)
    want = port.fixed(sample, L, L, idx.size, np.full(idx.size, init, dtype=np.uint32))
    if mask:
        want = np.array([port.mask(int(x)) for x in want], dtype=np.uint32)
    assert np.array_equal(long_[idx], want)


def test_fixed_dev_timed_matches_and_times(dev, C):
    n, L = 20000, 4096
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    C.fill_splitmix(buf, n, L, 0x5EED0001)
    plain = C.extend_fixed(buf, L, L, n).clone()
    b = C.FixedBatch(buf, L, L, n)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream(dev)
    e0.record(s)
    e1.record(s)
    for _ in range(3):
        b.launch_timed(e0, e1)
    torch.cuda.synchronize()
    assert torch.equal(b.out, plain)
    ms = e0.elapsed_time(e1)
    assert 0.0 < ms < 50.0, ms  # 82 MB: ~13 us at HBM rate; the kernel alone, not the queue


def test_host_paths_every_device_one_thread(dev, C, port):
    """One thread drives nvl_crc32c_batch_region_host / fixed_host on every
    visible device in turn; device indices >= the count are rejected."""
    from nvlevelz_amd import _lib
    ndev = torch.cuda.device_count()
    region = port.fill(0x4D, 0, 3_000_000)
    rng = np.random.default_rng(1)
    n = 500
    lens = rng.integers(0, 9000, n).astype(np.uint64)
    offs = (rng.random(n) * (region.nbytes - lens)).astype(np.uint64)
    want = [port.value(region[int(o):int(o) + int(m)].tobytes()) for o, m in zip(offs, lens)]
    try:
        for d in list(range(ndev)) * 2:
            torch.cuda.set_device(d)
            out = np.zeros(n, dtype=np.uint32)
            rc = _lib.lib.nvl_crc32c_batch_region_host(region.ctypes.data, region.nbytes, offs.ctypes.data,
                                                       lens.ctypes.data, None, 0, out.ctypes.data, n, 0)
            assert rc == 0, (d, rc)
            assert [int(x) for x in out] == want
            host = region[:700 * 4096]
            assert np.array_equal(C.extend_fixed_host(host, 4096, 4096, 700), port.fixed(host, 4096, 4096, 700))
    finally:
        torch.cuda.set_device(dev)
    assert _lib.lib.nvl_crc32c_init(ndev) == _lib.ENODEV
    assert _lib.lib.nvl_crc32c_init(64) == _lib.ENODEV
    assert _lib.lib.nvl_crc32c_init(-1) == _lib.ENODEV


def test_exiting_threads_release_device_memory(dev, C, port):
    """Each thread's fixed_host pipe holds two ~64 MiB device slabs and two
    streams; 40 short-lived threads must not leave 40 x 128 MiB behind."""
    host = port.fill(0x61, 0, 20000 * 4096)  # > one 64 MiB slab: both slabs in use
    want = port.fixed(host, 4096, 4096, 20000)
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(dev)
    errs = []

    def worker():
        try:
            torch.cuda.set_device(dev)
            if not np.array_equal(C.extend_fixed_host(host, 4096, 4096, 20000), want):
                errs.append("mismatch")
            C.extend_batch_host([host[:5000].tobytes()])
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))

    for _ in range(40):
        t = threading.Thread(target=worker)
        t.start()
        t.join()
    assert not errs
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info(dev)
    assert free0 - free1 < (1 << 30), (free0 - free1) / 2**20  # MiB retained
