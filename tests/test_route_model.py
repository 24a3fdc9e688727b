"""The routed calls' layout rule (crc32c_region.hip crc32c_route_plan,
modelled by tests/kernel_model.py route_plan_bad): what batch_dev accepts for
the region path must never make the region path read a 4 KiB page that holds
no buffer byte -- the only pages known to be mapped (buffers from different
allocations may have an unmapped page between them).  Checked against a
brute-force page cover over random sorted batches with gaps, empty buffers
and base alignments; the shapes of the call sites stay accepted."""
import numpy as np
import pytest

import kernel_model as km

NOLIM = (1 << 64) - 1


def _packed(lens, gaps, lead=0):
    lens = np.asarray(lens, dtype=np.int64)
    gaps = np.broadcast_to(np.asarray(gaps, dtype=np.int64), lens.shape)
    return lead + np.cumsum(lens + gaps) - lens - gaps


@pytest.mark.parametrize("seed", range(40))
def test_accepted_batches_touch_every_page(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 60))
    kind = seed % 4
    if kind == 0:  # gaps around a page
        gaps = rng.integers(0, 9000, n)
    elif kind == 1:  # mostly dense, a few page-sized gaps
        gaps = np.where(rng.random(n) < 0.2, rng.integers(4000, 4200, n), rng.integers(0, 8, n))
    elif kind == 2:  # empty buffers with small and large gaps
        gaps = np.where(rng.random(n) < 0.5, 0, rng.integers(0, 6000, n))
    else:
        gaps = rng.integers(0, 3, n)
    lens = np.where(rng.random(n) < 0.3, 0, rng.integers(1, 9000, n))
    base = int(rng.integers(0, 1 << 20)) << 12 | int(rng.integers(0, 4096))
    offs = _packed(lens, gaps, lead=int(rng.integers(0, 5000)))
    for _ in range(30):
        if not km.route_plan_bad(offs, lens, NOLIM, base, True):
            assert km.span_pages_touched(offs, lens, base), (offs, lens, base)
        # perturb: move one buffer's start, or empty / fill one
        j = int(rng.integers(0, n))
        if rng.random() < 0.5:
            lens = lens.copy()
            lens[j] = 0 if lens[j] else int(rng.integers(1, 5000))
        offs = _packed(lens, gaps, lead=int(offs[0]))


def test_page_rule_boundaries():
    """A buffer ending at a page end and the next starting one page later
    leaves a page untouched (rejected); starting in that page's last byte
    touches it (accepted).  An empty buffer may sit up to the end of the page
    of the previous buffer's last byte, not in the next one."""
    base = 7 << 12
    assert km.route_plan_bad([0, 8192], [4096, 10], NOLIM, base, True)
    assert not km.route_plan_bad([0, 8191], [4096, 10], NOLIM, base, True)
    assert not km.route_plan_bad([0, 4096], [4096, 10], NOLIM, base, True)
    # empty buffer right after the page of the last byte, then a buffer a page on
    assert not km.route_plan_bad([0, 4000, 4096], [10, 0, 10], NOLIM, base, True)
    assert not km.route_plan_bad([0, 4096, 4100], [4096, 0, 10], NOLIM, base, True)
    assert km.route_plan_bad([0, 4097, 8192], [10, 0, 10], NOLIM, base, True)
    assert km.route_plan_bad([0, 10], [0, 10], NOLIM, base, True)  # the first one empty
    assert not km.route_plan_bad([0, 10], [0, 10], NOLIM, base, False)  # region_dev: the caller's region
    # the base shifts pages: 4 bytes short of a page at base + 4092
    assert not km.route_plan_bad([0, 4000], [4, 10], NOLIM, base + 4092, True)  # next page
    assert km.route_plan_bad([0, 4100], [4, 10], NOLIM, base + 4092, True)  # one page further


def test_call_site_shapes_accepted():
    """The region path's intended batches stay on it: packed r / v / config 3
    shapes, SSTable block||type ranges (4-byte crc gaps), log records (7-byte
    headers, block padding)."""
    rng = np.random.default_rng(5)
    for lens, gaps, lead in (
            (rng.integers(3364, 4110, 3000), 4, 17),
            (np.full(2000, 4097), 0, 4093),
            (512 + rng.integers(0, 65025, 300), 0, 0),
            (rng.integers(1, 32768, 500), 7, 7),
            (rng.integers(1, 64, 5000), 0, 3)):
        offs = _packed(lens, gaps, lead)
        assert km.route_region_ok(offs, lens, NOLIM, 1 << 30, True, 36 * len(lens) + 20)
        assert km.route_region_ok(offs, lens, int(offs[-1] + lens[-1]), 1 << 30, False, 0)
    # sparse: 4 KiB buffers 1 MiB apart -> the page rule and the gap rule both say no
    lens = np.full(20, 4096)
    offs = _packed(lens, 1 << 20)
    assert km.route_plan_bad(offs, lens, NOLIM, 0, True)
    assert not km.route_plan_bad(offs, lens, NOLIM, 0, False)


def test_page_route_verdicts():
    """The page path takes what the region path does not, when every buffer
    is exactly 4096 bytes; a region-shaped batch of pages stays on the
    region path (it reads the same bytes, from one span)."""
    base = 1 << 30
    cap = lambda n: 36 * n + 20
    packed = 4096 * np.arange(64)
    assert km.route_verdict(packed, [4096] * 64, NOLIM, base, True, cap(64)) == "region"
    shuffled = packed[::-1]
    assert km.route_verdict(shuffled, [4096] * 64, NOLIM, base, True, cap(64)) == "pages_aligned"
    assert km.route_verdict(shuffled + 3, [4096] * 64, NOLIM, base, True, cap(64)) == "pages"
    far = 3 * packed  # sorted, gaps twice the bytes: the gap rule fails
    assert km.route_verdict(far, [4096] * 64, NOLIM, base, True, cap(64)) == "pages_aligned"
    over = 2048 * np.arange(64)  # overlapping
    assert km.route_verdict(over, [4096] * 64, NOLIM, base, True, cap(64)) == "pages_aligned"
    lens = [4096] * 64
    lens[7] = 4095
    assert km.route_verdict(shuffled, lens, NOLIM, base, True, cap(64)) == "heads"
    # region_dev (the caller's region): out of the region is not region-shaped
    assert km.route_verdict(packed, [4096] * 64, 4096 * 63, base, False, 0) == "pages_aligned"
