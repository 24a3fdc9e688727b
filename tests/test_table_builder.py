"""The SSTable writer shim against the reference's own TableBuilder.

oracle/ref_table.cc builds table/table_builder.cc, block_builder.cc,
filter_block.cc (+ util/bloom.cc) from /root/reference and drives one
key/value sequence through TableBuilder into (a) an in-memory WritableFile --
the reference's file -- and (b) a WritableFile that routes every block through
nvl::shims::TableFile (table_builder.cc:175-193 with the CRC deferred) and
seals all trailers in one engine batch.  The files must be byte-identical.

tests/golden/framing.json's "sstable_tables" are four such reference-built
tables (data, filter, metaindex and index blocks); they pin the seal and the
whole-table verify without the reference present (the GPU box)."""
import numpy as np
import pytest

import oracle
from conftest import gpu_present, load_golden
from nvlevelz_amd import framing

HOST = 0x100


def _cases(rng, count):
    for k in range(count):
        n = int(rng.integers(1, 600))
        keys = sorted({bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)) for _ in range(n)})
        vals = [bytes(rng.integers(0, 256, int(rng.integers(0, 700)), dtype=np.uint8)) for _ in keys]
        yield (keys, vals, int(rng.choice([64, 256, 1024, 4096, 16384])), int(rng.choice([1, 2, 16, 64])),
               int(rng.choice([0, 10])))


@pytest.mark.skipif(not oracle.ref_table_available(), reason="reference TableBuilder harness not built")
def test_tablefile_matches_reference_builder_live():
    rt = oracle.ref_table()
    rng = np.random.default_rng(1717)
    nblocks = 0
    for keys, vals, bs, ri, bloom in _cases(rng, 60):
        ref, _ = rt.build(keys, vals, bs, ri, bloom)
        img, hs = rt.build(keys, vals, bs, ri, bloom, via_shim=True, seal_flags=HOST)
        assert img == ref, (len(keys), bs, ri, bloom)
        rep = framing.verify_table(img, host=True)
        assert rep.ok and len(rep.blocks) >= 2
        nblocks += len(hs)
    assert nblocks > 300


def _zeroed(t):
    img = bytearray(bytes.fromhex(t["hex"]))
    for off, size in t["handles"]:
        img[off + size + 1:off + size + 5] = b"\0\0\0\0"
    return img


def _check_golden_tables(host):
    g = load_golden("framing")["sstable_tables"]
    assert len(g) == 4
    for t in g:
        want = bytes.fromhex(t["hex"])
        img = _zeroed(t)
        assert bytes(img) != want or not t["handles"]
        framing.seal_trailers(img, t["handles"], host=host)
        assert bytes(img) == want
        rep = framing.verify_table(want, host=host)
        assert rep.ok, rep
        v = framing.verify_blocks(want, t["handles"], host=host)
        assert (v == 0).all()


def test_golden_tables_host():
    _check_golden_tables(True)


@pytest.mark.gpu
def test_golden_tables_gpu():
    if not gpu_present():
        pytest.skip("no GPU")
    _check_golden_tables(False)


@pytest.mark.gpu
@pytest.mark.skipif(not oracle.ref_table_available(), reason="reference TableBuilder harness not built")
def test_tablefile_matches_reference_builder_gpu():
    if not gpu_present():
        pytest.skip("no GPU")
    rt = oracle.ref_table()
    rng = np.random.default_rng(1718)
    for keys, vals, bs, ri, bloom in _cases(rng, 20):
        ref, _ = rt.build(keys, vals, bs, ri, bloom)
        img, _ = rt.build(keys, vals, bs, ri, bloom, via_shim=True, seal_flags=0)
        assert img == ref, (len(keys), bs, ri, bloom)
