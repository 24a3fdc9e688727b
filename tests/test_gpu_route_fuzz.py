"""Randomised routed calls: 400 batches of random shape --
sorted and dense, sorted with gaps (some over a page), unsorted, overlapping,
with empty buffers, long buffers over the 128 KiB limit, tiny and large n,
exactly-4096-byte buffers anywhere (the page path) --
through nvl_crc32c_batch_dev and nvl_crc32c_region_dev on one stream and ONE
reused workspace, every CRC against the oracle.  Back-to-back calls of
different layouts share the workspace's plan partials and event records, so
a verdict or a record left over from an earlier call would show here.
Sorted, non-overlapping batches also run with NVL_CRC32C_FLAG_REGION_SHAPED
(the one-launch region kernel) on the same workspace.  NVL_FUZZ_ITERS /
NVL_FUZZ_SEED widen the run (a stress pass; the suite runs 400 from seed 2026)."""
import os

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


def _t64(a, dev):
    return torch.from_numpy(np.asarray(a, dtype=np.uint64).view(np.int64)).to(dev)


def _batch(rng, image):
    kind = int(rng.integers(0, 7))
    n = int(rng.choice([1, 2, 7, 63, 64, 65, 500, 3000, 20_000, 70_000]))
    if kind == 6:  # exactly-4096-byte buffers anywhere (the page path unless region-shaped): random
        # positions on a 4 KiB, 16-byte or 1-byte grid -- in any order, overlapping -- or packed
        g = int(rng.choice([4096, 16, 1]))
        if rng.random() < 0.2:
            offs = 4096 * np.arange(min(n, image // 4096 - 1)) + int(rng.integers(0, 64)) * g % 4096
        else:
            offs = rng.integers(0, (image - 4096) // g, n) * g
        return offs.astype(np.int64), np.full(len(offs), 4096, dtype=np.int64), False
    if kind == 4:  # long buffers, some over the region path's 128 KiB limit
        lens = rng.integers(1, 300_000, n)
    elif kind == 5:  # tiny
        lens = rng.integers(0, 70, n)
    else:
        lens = rng.integers(0, 9000, n)
    gaps = np.where(rng.random(n) < 0.05, rng.integers(0, 12_000, n), rng.integers(0, 8, n))
    offs = np.cumsum(lens + gaps) - lens - gaps + int(rng.integers(0, 4096))
    if offs[-1] + lens[-1] > image:  # fit the image: scale down
        keep = max(1, int(np.searchsorted(offs + lens, image)) - 1)
        offs, lens = offs[:keep], lens[:keep]
    if kind == 1:  # unsorted
        p = rng.permutation(len(offs))
        offs, lens = offs[p], lens[p]
    elif kind == 2 and len(offs) > 1:  # overlapping: some starts pulled back
        j = rng.integers(1, len(offs), max(1, len(offs) // 50))
        offs = offs.copy()
        offs[j] = np.maximum(0, offs[j] - rng.integers(1, 5000, j.size))
    return offs.astype(np.int64), lens.astype(np.int64), kind in (0, 3, 4, 5)


def test_random_routed_batches(dev, port):
    from nvlevelz_amd import crc32c as C
    rng = np.random.default_rng(int(os.environ.get("NVL_FUZZ_SEED", "2026")))
    image = 96 << 20
    host = port.fill(0xF022, 0, image)
    buf = torch.from_numpy(host).to(dev)
    wsb = max(C.batch_workspace_bytes(70_000), C.region_workspace_bytes(image, 70_000))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    for it in range(int(os.environ.get("NVL_FUZZ_ITERS", "400"))):
        offs, lens, sorted_ = _batch(rng, image)
        n = len(offs)
        inits = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), inits)
        ti = torch.from_numpy(inits.view(np.int32)).to(dev)
        o, m = _t64(offs, dev), _t64(lens, dev)
        f = C.extend_batch if it % 2 == 0 else C.extend_region
        got = f(buf, o, m, ti, workspace=ws).cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (it, f.__name__, n, bad[:5], offs[bad[:5]], lens[bad[:5]])
        if sorted_ and it % 3 == 0:  # the caller's promise kept: one region-kernel launch
            got = C.extend_region(buf, o, m, ti, workspace=ws, shaped=True).cpu().numpy().view(np.uint32)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (it, "shaped", n, bad[:5], offs[bad[:5]], lens[bad[:5]])
