"""The oracle (CPU restatement, oracle/crc32c_oracle.c) pinned against the
reference-generated golden vectors (tests/golden/, made by
oracle/gen_golden.py from the reference's own util/crc32c.cc +
port/port_posix_sse.cc) and, when oracle/_ref is built, against the
reference objects directly.  CPU only."""
import numpy as np
import pytest

import oracle
from conftest import load_golden


def aligned(nbytes, align=4096):
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


# util/crc32c_test.cc:13-48 (RFC 3720 B.4) + extra reference KATs
def test_kat_values(port):
    g = load_golden("kat")
    for v in g["value"]:
        data = bytes.fromhex(v["hex"])
        assert port.value(data) == v["crc"], v["name"]
        assert port.extend_table(0, data) == v["crc"], v["name"]
        assert port.extend_sse(0, data) in (v["crc"], 0), v["name"]  # 0 = no SSE4.2 (port_example.h:132-136)


def test_rfc3720_literals(port):
    # the literal constants of util/crc32c_test.cc:18-47
    assert port.value(bytes(32)) == 0x8A9136AA
    assert port.value(b"\xff" * 32) == 0x62A8AB43
    assert port.value(bytes(range(32))) == 0x46DD794E
    assert port.value(bytes(range(31, -1, -1))) == 0x113FDB5C


def test_kat_extend_and_mask(port):
    g = load_golden("kat")
    for e in g["extend"]:
        assert port.extend(e["init"], bytes.fromhex(e["hex"])) == e["crc"]
    for m in g["mask"]:
        assert port.mask(m["crc"]) == m["masked"]
        assert port.unmask(m["crc"]) == m["unmasked"]
        assert port.unmask(port.mask(m["crc"])) == m["crc"]


def test_crc32c_test_properties(port):
    # util/crc32c_test.cc:50-65
    assert port.value(b"a") != port.value(b"foo")
    assert port.value(b"hello world") == port.extend(port.value(b"hello "), b"world")
    crc = port.value(b"foo")
    assert crc != port.mask(crc)
    assert crc != port.mask(port.mask(crc))
    assert crc == port.unmask(port.mask(crc))
    assert crc == port.unmask(port.unmask(port.mask(port.mask(crc))))


def test_probe_constant(port):
    # util/crc32c.cc:290-297
    assert port.value(b"TestCRCBuffer") == 0xDCBC59FA


@pytest.mark.parametrize("which", ["extend", "extend_table"])
def test_sweep_golden(port, which):
    g = load_golden("sweep")
    buf = aligned(g["stream_bytes"])
    buf[:] = port.fill(g["seed"], 0, buf.size)
    f = getattr(port.lib, "oracle_crc32c_" + which)
    for oi, o in enumerate(g["offsets"]):
        got = [f(0, buf.ctypes.data + o, n) for n in g["lengths"]]
        assert got == g["crc"][oi], (which, o)
    for o, n, init, crc in g["extend"]:
        assert f(init, buf.ctypes.data + o, n) == crc


def test_framing_golden(port):
    g = load_golden("framing")
    for b in g["sstable_blocks"]:
        data = bytes.fromhex(b["hex"])
        # table/table_builder.cc:185-187
        crc = port.extend(port.value(data), bytes([b["type"]]))
        assert crc == b["crc"] and port.mask(crc) == b["masked"]
        # table/format.cc:90-92 checks Value(data, n+1) == Unmask(stored)
        assert port.value(data + bytes([b["type"]])) == port.unmask(b["masked"]) == b["check"]
    for r in g["log_records"]:
        payload = port.fill(r["seed"], 0, r["len"]).tobytes()
        # db/log_writer.cc:15-20,95-96 and db/log_reader.cc:255-256
        assert port.value(bytes([r["type"]])) == r["type_crc"]
        crc = port.extend(r["type_crc"], payload)
        assert crc == r["crc"] and port.mask(crc) == r["masked"]
        assert port.value(bytes([r["type"]]) + payload) == r["crc"]


def test_config2_golden(port):
    g = load_golden("configs")["cfg2"]
    n, L = g["n"], g["len"]
    buf = port.fill(g["seed"], 0, n * L)
    crc = port.fixed_mt(buf, L, L, n, 8)
    assert [int(x) for x in crc[:8]] == g["crc_first"]
    assert int(crc[-1]) == g["crc_last"]
    assert port.digest(crc) == g["digest"]
    assert np.array_equal(port.fixed(buf[:4096 * 64], L, L, 64), crc[:64])


def test_config3_golden(port):
    g = load_golden("configs")["cfg3"]
    lens = port.cfg3_lengths(g["len_seed"], g["total"])
    assert lens.size == g["n"] and lens[0] == g["len_first"] and lens[-1] == g["len_last"]
    assert int(lens.sum()) == g["total"]
    buf = port.fill(g["seed"], 0, g["total"])
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    crc = port.varlen(buf, offs, lens)
    assert [int(x) for x in crc[:8]] == g["crc_first"]
    assert int(crc[-1]) == g["crc_last"]
    assert port.digest(crc) == g["digest"]


@pytest.mark.slow
def test_config4_golden_streamed(port):
    g = load_golden("configs")["cfg4"]
    n, L = g["n"], g["len"]
    crc = np.empty(n, dtype=np.uint32)
    step = 250
    for s in range(0, n, step):
        part = port.fill(g["seed"], s * L, step * L)
        crc[s:s + step] = port.fixed_mt(part, L, L, step, 8)
    assert [int(x) for x in crc[:8]] == g["crc_first"]
    assert int(crc[-1]) == g["crc_last"]
    assert port.digest(crc) == g["digest"]


def test_fill_is_splitmix64(port):
    # SURVEY.md §8d definition, restated in numpy
    seed = 0x5EED0001
    k = np.arange(1, 9, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    assert np.array_equal(port.fill(seed, 0, 64), z.view(np.uint8))
    assert np.array_equal(port.fill(seed, 13, 30), z.view(np.uint8)[13:43])


@pytest.mark.skipif(not oracle.ref_available("sse") or not oracle.ref_available("table"),
                    reason="oracle/_ref not built")
def test_port_matches_reference_objects(port):
    """The restatement against the reference compiled from /root/reference."""
    rs, rt = oracle.ref("sse"), oracle.ref("table")
    rng = np.random.default_rng(42)
    buf = aligned(1 << 17)
    buf[:] = rng.integers(0, 256, buf.size, dtype=np.uint8)
    for _ in range(3000):
        o = int(rng.integers(0, 4096))
        n = int(rng.integers(0, 20000))
        init = int(rng.integers(0, 2**32))
        want = rs.extend_at(init, buf, o, n)
        assert rt.extend_at(init, buf, o, n) == want
        assert port.lib.oracle_crc32c_extend(init, buf.ctypes.data + o, n) == want
        assert port.lib.oracle_crc32c_extend_table(init, buf.ctypes.data + o, n) == want
    assert rs.mask(0x12345678) == port.mask(0x12345678)
    assert rs.unmask(0x12345678) == port.unmask(0x12345678)
