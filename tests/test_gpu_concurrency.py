"""Concurrent callers (SURVEY §8b threading: the fork calls Extend from
foreground readers, the compaction thread and MANIFEST writers at once,
util/env_posix.cc:911-952, db/version_set.cc:901-909): host threads, each on
its own stream, interleave every entry kind that keeps per-thread or
per-stream state -- routed and shaped region batches (the stream's counter
block, the call generation), the batch path on shuffled blocks, the
device-resident whole-table verify (the thread's table workspace, side
stream, pinned buffers) and the host region entry from registered and
unregistered memory (the thread's staging and result buffers).  Every result
is checked against the oracle or against the same call made alone."""
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# (NVL_CONC_THREADS / NVL_CONC_ITERS widen it for a stress pass)
THREADS = int(os.environ.get("NVL_CONC_THREADS", "4"))
ITERS = int(os.environ.get("NVL_CONC_ITERS", "5"))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from nvlevelz_amd import crc32c
    d = torch.device("cuda:0")
    torch.cuda.set_device(d)
    crc32c.init(0)
    return d


def _u32(t):
    return t.detach().cpu().numpy().view(np.uint32)


def test_concurrent_entry_kinds(dev, port):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from nvlevelz_amd import crc32c, framing

    # per thread: an `r`-shaped region batch, a shuffled 4 KiB batch, a host region
    cases = []
    for k in range(THREADS):
        rng = np.random.default_rng(900 + k)
        lens = rng.integers(3364, 4110, 2500 + 300 * k).astype(np.int64)
        offs = (np.cumsum(lens + 4) - lens - 4).astype(np.int64)
        host = port.fill(0xC0 + k, 0, int(offs[-1] + lens[-1]) + 64)
        inits = rng.integers(0, 2**32, size=lens.size, dtype=np.uint64).astype(np.uint32)
        want = port.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64), inits)
        nb = 1500
        perm = rng.permutation(nb).astype(np.int64) * 4096
        hb = port.fill(0xD0 + k, 0, nb * 4096)
        want_b = port.varlen(hb, perm.astype(np.uint64), np.full(nb, 4096, dtype=np.uint64))
        reg = np.ascontiguousarray(host.copy())
        cases.append(dict(lens=lens, offs=offs, host=host, inits=inits, want=want, perm=perm, hb=hb,
                          want_b=want_b, reg=reg))
    image = bench.build_table_image(300 + 0, 4096)
    dimg = torch.frombuffer(bytearray(image), dtype=torch.uint8).to(dev)
    ref_report = framing.verify_table_dev(dimg)
    assert ref_report.ok
    ref_blocks = [(b.offset, b.size, b.role, b.verdict) for b in ref_report.blocks]
    for c in cases:
        crc32c.host_register(c["reg"])
    errs = []

    def worker(k):
        c = cases[k]
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                buf = torch.from_numpy(c["host"]).to(dev)
                o = torch.from_numpy(c["offs"]).to(dev)
                m = torch.from_numpy(c["lens"]).to(dev)
                it = torch.from_numpy(c["inits"].view(np.int32)).to(dev)
                bb = torch.from_numpy(c["hb"]).to(dev)
                bo = torch.from_numpy(c["perm"]).to(dev)
                bm = torch.full((c["perm"].size,), 4096, dtype=torch.int64, device=dev)
                for i in range(ITERS):
                    r1 = crc32c.extend_region(buf, o, m, it)                 # routed (plan, route, body)
                    r2 = crc32c.extend_region(buf, o, m, it, shaped=True)    # one region launch
                    r3 = crc32c.extend_batch(bb, bo, bm)                      # not region-shaped: page path
                    s.synchronize()
                    for name, got, want in (("routed", r1, c["want"]), ("shaped", r2, c["want"]),
                                            ("batch", r3, c["want_b"])):
                        if not np.array_equal(_u32(got), want):
                            errs.append((k, i, name))
                    rep = framing.verify_table_dev(dimg, stream=s.cuda_stream)
                    if not rep.ok or [(b.offset, b.size, b.role, b.verdict) for b in rep.blocks] != ref_blocks:
                        errs.append((k, i, "table_dev"))
                    src = c["reg"] if i % 2 == 0 else c["host"]              # registered, then staged
                    h = crc32c.extend_region_host(src, c["offs"], c["lens"], c["inits"])
                    if not np.array_equal(np.asarray(h, dtype=np.uint32), c["want"]):
                        errs.append((k, i, "host_region", i % 2 == 0))
        except Exception as e:  # pragma: no cover
            errs.append((k, repr(e)))

    try:
        th = [threading.Thread(target=worker, args=(k,)) for k in range(THREADS)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        torch.cuda.synchronize()
        for c in cases:
            crc32c.host_unregister(c["reg"])
    assert not errs, errs[:10]
