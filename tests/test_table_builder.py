"""The SSTable writer shim against the reference's own TableBuilder.

oracle/ref_table.cc builds table/table_builder.cc, block_builder.cc,
filter_block.cc (+ util/bloom.cc) from /root/reference and drives one
key/value sequence through TableBuilder into (a) an in-memory WritableFile --
the reference's file -- and (b) the shipped adapter
nvl::shims::BatchingWritableFile<leveldb::WritableFile, leveldb::Slice,
leveldb::Status> around it (include/nvl_leveldb_shims.h), which stages every
block with a placeholder trailer and seals the trailers in engine batches (at
Close, or every ~5000 staged bytes).  The files must be byte-identical.

The same harness is built a second time with INTEGRATION.md §5's edit of
WriteRawBlock applied at build time (oracle/apply_deferred_crc.py): there the
reference computes no block CRC at all when its file is the adapter -- the
staged trailers hold zero CRCs -- and the sealed file is still identical.

tests/golden/framing.json's "sstable_tables" are four such reference-built
tables (data, filter, metaindex and index blocks); they pin the seal and the
whole-table verify without the reference present (the GPU box)."""
import numpy as np
import pytest

import oracle
from conftest import gpu_present, load_golden
from nvlevelz_amd import framing

HOST = 0x100
GPU = 0x400  # NVL_FRAMING_GPU


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
        img, hs = rt.build(keys, vals, bs, ri, bloom, via_shim=1, seal_flags=HOST)
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
        img, _ = rt.build(keys, vals, bs, ri, bloom, via_shim=1, seal_flags=GPU)
        assert img == ref, (len(keys), bs, ri, bloom)


def _trailer_crcs(img, hs):
    return [bytes(img[o + sz + 1:o + sz + 5]) for o, sz in hs]


@pytest.mark.skipif(not (oracle.ref_table_available() and oracle.ref_table_available(deferred=True)),
                    reason="reference TableBuilder harnesses not built")
def test_batching_file_and_deferred_crc_edit_live():
    """The adapter sealing at Close and every ~5000 bytes, around the stock
    and the edited TableBuilder: byte-identical files; with the edit the
    staged trailers carry no CRC (the reference computed none)."""
    stock, edited = oracle.ref_table(), oracle.ref_table(deferred=True)
    rng = np.random.default_rng(1719)
    multi = 0
    for keys, vals, bs, ri, bloom in _cases(rng, 40):
        ref, _ = stock.build(keys, vals, bs, ri, bloom)
        for rt in (stock, edited):
            for mode in (1, 2):
                img, hs = rt.build(keys, vals, bs, ri, bloom, via_shim=mode, seal_flags=HOST)
                assert img == ref, (rt.path, mode, len(keys), bs)
                if mode == 2:
                    multi += rt.seals > 1
        assert edited.build(keys, vals, bs, ri, bloom)[0] == ref  # a plain file: the edit computes the CRCs
        staged_e, hs_e = edited.build(keys, vals, bs, ri, bloom, via_shim=3, seal_flags=HOST)
        computed_e = edited.computed
        staged_s, hs_s = stock.build(keys, vals, bs, ri, bloom, via_shim=3, seal_flags=HOST)
        assert hs_e == hs_s and hs_e
        assert staged_e == staged_s  # placeholders either way
        assert all(c == b"\0\0\0\0" for c in _trailer_crcs(staged_e, hs_e))
        # the stock builder computed (nearly) every block's CRC, the edited one none
        assert computed_e == 0 and stock.computed >= len(hs_s) - 1
    assert multi > 10


@pytest.mark.gpu
@pytest.mark.skipif(not oracle.ref_table_available(deferred=True), reason="reference TableBuilder harness not built")
def test_deferred_crc_edit_gpu_seal():
    if not gpu_present():
        pytest.skip("no GPU")
    stock, edited = oracle.ref_table(), oracle.ref_table(deferred=True)
    rng = np.random.default_rng(1720)
    for keys, vals, bs, ri, bloom in _cases(rng, 10):
        ref, _ = stock.build(keys, vals, bs, ri, bloom)
        for mode in (1, 2):
            img, _ = edited.build(keys, vals, bs, ri, bloom, via_shim=mode, seal_flags=GPU)
            assert img == ref, (mode, len(keys), bs)
