#!/usr/bin/env python3
"""Generate tests/golden/*.json from the REFERENCE's own CRC32C build.

TEST INFRASTRUCTURE.  Runs in the build container only (needs
oracle/_ref/libref_crc32c_{sse,table}.so, i.e. util/crc32c.cc +
port/port_posix_sse.cc compiled from /root/reference by oracle/Makefile).
Every expected value below is produced by calling the reference's
leveldb::crc32c::Extend / Value / Mask / Unmask, and cross-checked between
the SSE4.2 build (port/port_posix_sse.cc:69-126) and the table build
(util/crc32c.cc:305-346) before it is written.  The inputs are either the
RFC 3720 vectors from util/crc32c_test.cc:13-65 or the canonical splitmix64
stream of SURVEY.md §8d.

    python oracle/gen_golden.py            # writes tests/golden/
    python oracle/gen_golden.py --no-cfg4  # skip the 10 GiB config-4 pass
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "tests", "golden")


def both(fn):
    """Evaluate fn(ref_lib) on both reference builds and require agreement."""
    a = fn(oracle.ref("sse"))
    b = fn(oracle.ref("table"))
    assert a == b, (a, b)
    return a


def aligned_buffer(nbytes: int, align: int = 4096) -> np.ndarray:
    raw = np.zeros(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def kat() -> dict:
    out = {"source": "util/crc32c_test.cc:13-65 + extra reference calls", "value": [], "extend": [],
           "mask": []}

    def add_value(name, data: bytes):
        out["value"].append({"name": name, "hex": data.hex(),
                             "crc": both(lambda r: r.value(data))})

    add_value("rfc3720_zeros32", bytes(32))
    add_value("rfc3720_ones32", b"\xff" * 32)
    add_value("rfc3720_inc32", bytes(range(32)))
    add_value("rfc3720_dec32", bytes(range(31, -1, -1)))
    add_value("rfc3720_iscsi48", bytes([
        0x01, 0xc0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
        0x14, 0, 0, 0, 0, 0, 0x04, 0, 0, 0, 0, 0x14, 0, 0, 0, 0x18,
        0x28, 0, 0, 0, 0, 0, 0, 0, 0x02, 0, 0, 0, 0, 0, 0, 0]))
    add_value("check_123456789", b"123456789")
    add_value("empty", b"")
    add_value("a", b"a")
    add_value("foo", b"foo")
    add_value("hello world", b"hello world")
    add_value("TestCRCBuffer", b"TestCRCBuffer")
    add_value("x4096", b"x" * 4096)  # db/db_bench.cc:729-746 input

    def add_extend(init, data: bytes):
        out["extend"].append({"init": init, "hex": data.hex(),
                              "crc": both(lambda r: r.extend(init, data))})

    add_extend(0x12345678, b"")
    add_extend(both(lambda r: r.value(b"hello ")), b"world")
    add_extend(0xFFFFFFFF, b"abc")
    add_extend(0xDEADBEEF, bytes(range(256)) * 3)
    for v in [0, 1, 0xFFFFFFFF, 0x12345678, 0xdcbc59fa, 0x80000000, 0xa282ead8]:
        out["mask"].append({"crc": v, "masked": both(lambda r: r.mask(v)),
                            "unmasked": both(lambda r: r.unmask(v))})
    return out


def sweep() -> dict:
    """CRCs of stream bytes at every (offset 0..15, length 0..320) plus a few
    long lengths, each evaluated at its true address alignment (offset o within
    a 4096-aligned buffer) so both reference backends' alignment prologues are
    exercised."""
    seed = 0x5EED00AA
    p = oracle.port()
    buf = aligned_buffer(70000)
    buf[:] = p.fill(seed, 0, buf.size)
    lengths = list(range(0, 321)) + [511, 512, 513, 1023, 1024, 1025, 4095, 4096, 4097,
                                     4100, 8191, 8192, 12345, 65535, 65536]
    crcs = []
    for o in range(16):
        row = []
        for n in lengths:
            row.append(both(lambda r: r.extend_at(0, buf, o, n)))
        crcs.append(row)
    # Extend() with non-zero init at a handful of (offset, length) points
    rng = np.random.default_rng(1234)
    ext = []
    for _ in range(200):
        o = int(rng.integers(0, 4096))
        n = int(rng.integers(0, 9000))
        init = int(rng.integers(0, 2**32))
        ext.append([o, n, init, both(lambda r: r.extend_at(init, buf, o, n))])
    return {"seed": seed, "stream_bytes": int(buf.size), "offsets": list(range(16)),
            "lengths": lengths, "crc": crcs, "extend": ext}


def framing() -> dict:
    """SSTable block trailers (table/table_builder.cc:183-188, checked by
    table/format.cc:90-96) and log record headers (db/log_writer.cc:88-97,
    checked by db/log_reader.cc:253-256) for synthetic contents, plus whole
    tables written by the reference's own TableBuilder."""
    p = oracle.port()
    rng = np.random.default_rng(99)
    blocks = []
    for i in range(12):
        n = int(rng.integers(3363, 4109))  # data-block sizes measured in SURVEY §3A
        data = p.fill(0x5EED00B0 + i, 0, n).tobytes()
        btype = int(i % 2)  # kNoCompression=0, kSnappyCompression=1
        crc = both(lambda r: r.extend(r.value(data), bytes([btype])))
        blocks.append({"hex": data.hex(), "type": btype, "crc": crc,
                       "masked": both(lambda r: r.mask(crc)),
                       "check": both(lambda r: r.value(data + bytes([btype])))})
    records = []
    for i in range(12):
        n = int(rng.integers(0, 32762))  # kBlockSize - kHeaderSize payload cap
        payload = p.fill(0x5EED00C0 + i, 0, n).tobytes()
        rtype = int(1 + i % 4)  # kFullType..kLastType
        type_crc = both(lambda r: r.value(bytes([rtype])))
        crc = both(lambda r: r.extend(type_crc, payload))
        records.append({"len": n, "seed": 0x5EED00C0 + i, "type": rtype, "type_crc": type_crc,
                        "crc": crc, "masked": both(lambda r: r.mask(crc))})
    # Real tables: the reference's TableBuilder (oracle/ref_table.cc) over
    # deterministic key/value sets; every block (data, filter, metaindex,
    # index) with its handle, and the real data blocks appended to
    # sstable_blocks as well.
    tables = []
    if oracle.ref_table_available():
        rt = oracle.ref_table()
        for ti, (n, bs, ri, bloom) in enumerate([(300, 1024, 16, 0), (400, 4096, 4, 10), (1, 4096, 16, 0),
                                                 (120, 256, 1, 10)]):
            keys = [b"key%08d" % (i * 7 + ti) for i in range(n)]
            vals = [p.fill(0x7AB1E000 + ti * 1000 + i, 0, int(rng.integers(0, 300))).tobytes() for i in range(n)]
            img, _ = rt.build(keys, vals, bs, ri, bloom)
            img2, hs = rt.build(keys, vals, bs, ri, bloom, via_shim=True, seal_flags=0x100)
            assert img2 == img, "TableFile seal differs from the reference TableBuilder"
            tables.append({"entries": n, "block_size": bs, "restart_interval": ri, "bloom_bits": bloom,
                           "hex": img.hex(), "handles": hs, "image_crc": both(lambda r: r.value(img))})
            if ti == 1:
                for (o, sz) in hs:
                    data = img[o:o + sz]
                    btype = img[o + sz]
                    crc = both(lambda r: r.extend(r.value(data), bytes([btype])))
                    blocks.append({"hex": data.hex(), "type": btype, "crc": crc, "masked": both(lambda r: r.mask(crc)),
                                   "check": both(lambda r: r.value(data + bytes([btype]))),
                                   "source": "TableBuilder (oracle/ref_table.cc), table 1"})
    return {"sstable_blocks": blocks, "log_records": records, "sstable_tables": tables}


def log_cases() -> dict:
    """Log scenarios (tests/framing_cases.py) run through the REFERENCE's own
    log::Writer (db/log_writer.cc) and log::Reader (db/log_reader.cc), built
    from /root/reference into oracle/_ref/libref_framing.so."""
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN)))
    import framing_cases as fc  # tests/framing_cases.py
    p = oracle.port()
    rf = oracle.ref_framing()
    cases = []
    for spec in fc.named() + fc.random_cases(300):
        img = fc.write_image(p, spec, rf.log_write)
        muts, io = fc.resolve(p, spec, img)
        bad = fc.mutate(p, img, muts)
        trace = rf.log_read(bad, spec["checksum"], io)
        c = dict(spec)
        c.update({"image_len": len(img), "image_crc": p.value(img), "mutations": muts,
                  "initial_offset": io, "read_len": len(bad), "read_crc": p.value(bad)})
        c.pop("mutations_rel", None)
        c.pop("initial_offset_rel", None)
        if len(trace) <= 6000:
            c["trace"] = trace
        else:
            c["trace_crc"] = p.value(trace.encode())
            c["trace_lines"] = trace.count("\n")
        cases.append(c)
    return {"cases": cases}


def configs(do_cfg4: bool) -> dict:
    p = oracle.port()
    r = oracle.ref("sse")
    out = {}
    # config 2: 1e5 x 4096, stride 4096, seed 0x5EED0001
    n, L = 100_000, 4096
    buf = aligned_buffer(n * L)
    buf[:] = p.fill(0x5EED0001, 0, buf.size)
    crc = r.fixed_mt(buf, L, L, n, 8)
    assert crc[0] == oracle.ref("table").value(buf[:L].tobytes())
    out["cfg2"] = {"seed": 0x5EED0001, "n": n, "len": L, "stride": L,
                   "crc_first": [int(x) for x in crc[:8]], "crc_last": int(crc[-1]),
                   "digest": p.digest(crc)}
    del buf
    # config 3: 1 GiB packed variable lengths
    total = 1 << 30
    lens = p.cfg3_lengths(0x5EED0003, total)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    buf = aligned_buffer(total)
    buf[:] = p.fill(0x5EED0002, 0, total)
    crc = np.array([r.extend_at(0, buf, int(o), int(m)) for o, m in zip(offs, lens)],
                   dtype=np.uint32)
    out["cfg3"] = {"seed": 0x5EED0002, "len_seed": 0x5EED0003, "total": total,
                   "n": int(lens.size), "len_first": int(lens[0]), "len_last": int(lens[-1]),
                   "crc_first": [int(x) for x in crc[:8]], "crc_last": int(crc[-1]),
                   "digest": p.digest(crc)}
    del buf
    if do_cfg4:
        n, L = 5000, 2 << 20
        crc = np.empty(n, dtype=np.uint32)
        part = aligned_buffer(L * 100)
        for s in range(0, n, 100):
            part[:] = p.fill(0x5EED0004, s * L, part.size)
            crc[s:s + 100] = r.fixed_mt(part, L, L, 100, 8)
        out["cfg4"] = {"seed": 0x5EED0004, "n": n, "len": L, "stride": L,
                       "crc_first": [int(x) for x in crc[:8]], "crc_last": int(crc[-1]),
                       "digest": p.digest(crc)}
    return out


def cfg5() -> dict:
    """Config 5 (BASELINE.json configs[4]): 10^7 x 4096 B of the splitmix64
    stream seeded 0x5EED0005, buffer i = stream bytes [4096 i, 4096 i + 4096)
    (buffer i lives on GPU i mod G, generated in place there).
    41 GB never fits here at once: the stream is generated in 10^5-block
    chunks and checksummed by the oracle's C restatement (oracle/crc32c_oracle.c,
    the port of port/port_posix_sse.cc:69-126).  The restatement is pinned
    first: the 10^5-block prefix (and every 10th chunk) is also checksummed by
    the REFERENCE's own build (oracle/_ref, util/crc32c.cc +
    port/port_posix_sse.cc) and must agree CRC for CRC.  The digest is
    Value() over the little-endian array of all 10^7 CRCs in global order,
    the same definition as configs 2-4.  Per-10^6-block sub-digests are kept
    too, so a shard test can check a part without the whole."""
    p = oracle.port()
    r = oracle.ref("sse")
    n, L, chunk = 10_000_000, 4096, 100_000
    th = min(8, os.cpu_count() or 1)
    crc = np.empty(n, dtype=np.uint32)
    part = aligned_buffer(chunk * L)
    ref_checked = 0
    for k, s in enumerate(range(0, n, chunk)):
        part[:] = p.fill(0x5EED0005, s * L, part.size)
        crc[s:s + chunk] = p.fixed_mt(part, L, L, chunk, th)
        if k % 10 == 0:
            want = r.fixed_mt(part, L, L, chunk, th)
            assert np.array_equal(crc[s:s + chunk], want), f"restatement != reference on chunk {k}"
            ref_checked += chunk
    sub = [p.digest(crc[s:s + 1_000_000]) for s in range(0, n, 1_000_000)]
    # bench.py --gpus N's cfg5 leg: rank r holds blocks r, r + N, ... (round
    # robin); each rank checks its own digest over its CRCs in local order
    # (shard.verify_shards), rank 0 the gathered global one
    ranks = {str(N): {"rank_digests": [p.digest(crc[k::N]) for k in range(N)]} for N in (2, 3, 4, 8)}
    return {"seed": 0x5EED0005, "n": n, "len": L, "stride": L,
            "crc_first": [int(x) for x in crc[:8]], "crc_last": int(crc[-1]),
            "digest": p.digest(crc), "sub_digest_blocks": 1_000_000, "sub_digests": [int(x) for x in sub],
            "ranks": ranks, "ref_checked_blocks": ref_checked,
            "how": "oracle restatement (port) over all blocks; reference build (oracle/_ref) on every 10th "
                   "10^5-block chunk incl. the prefix, identical; ranks[N].rank_digests = Value() over "
                   "rank r's CRCs (blocks r, r+N, ...) in local order"}


def cfg2_union() -> dict:
    """Config 2 at N GPUs (bench.py's weak scaling: 10^5 blocks PER rank,
    rank r holding global blocks r, r + N, r + 2N, ...): the union is global
    blocks 0 .. N*10^5 - 1 of the config-2 stream (seed 0x5EED0001).  For N =
    2, 4 and 8: the digest of all N*10^5 CRCs in global order (what rank 0
    checks after shard.gather_crcs) and each rank's own digest over its
    blocks in local order (what every rank checks by itself).  CRCs by the
    REFERENCE's own build (oracle/_ref), in 10^5-block slices."""
    p = oracle.port()
    r = oracle.ref("sse")
    per, L, nmax = 100_000, 4096, 8
    th = min(8, os.cpu_count() or 1)
    crc = np.empty(per * nmax, dtype=np.uint32)
    part = aligned_buffer(per * L)
    for s in range(0, per * nmax, per):
        part[:] = p.fill(0x5EED0001, s * L, part.size)
        crc[s:s + per] = r.fixed_mt(part, L, L, per, th)
    out = {"seed": 0x5EED0001, "blocks_per_rank": per, "len": L,
           "how": "reference build (oracle/_ref, util/crc32c.cc + port/port_posix_sse.cc) over global blocks "
                  "0 .. 8*10^5-1; digest = Value() of the little-endian CRC array"}
    for N in (2, 4, 8):
        u = crc[:per * N]
        out[str(N)] = {"digest": p.digest(u), "crc_last": int(u[-1]),
                       "rank_digests": [p.digest(u[k::N]) for k in range(N)]}
    return out


def table_cases() -> dict:
    """SSTable scenarios (tests/table_cases.py) scanned by the REFERENCE's own
    Footer::DecodeFrom, ReadBlock and Block::Iter (table/format.cc,
    table/block.cc) through oracle/ref_framing.cc:ref_table_scan."""
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN)))
    import table_cases as tc  # tests/table_cases.py
    p = oracle.port()
    rf = oracle.ref_framing()
    cases = []
    for spec in tc.named() + tc.random_cases(300):
        img, _ = tc.build(p, spec)
        c = dict(spec)
        c.update({"image_len": len(img), "image_crc": p.value(img), "trace": rf.table_scan(img)})
        cases.append(c)
    return {"cases": cases}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-cfg4", action="store_true")
    ap.add_argument("--only", default="", help="comma list of fixtures to regenerate (kat,sweep,framing,log_cases,table_cases,configs)")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    os.makedirs(GOLDEN, exist_ok=True)
    provenance = {"generator": "oracle/gen_golden.py",
                  "reference_builds": [oracle.ref("sse").path, oracle.ref("table").path,
                                       os.path.join(os.path.dirname(oracle.ref("sse").path), "libref_framing.so"),
                                       os.path.join(os.path.dirname(oracle.ref("sse").path), "libref_table.so")]}
    for name, fn in [("kat", kat), ("sweep", sweep), ("framing", framing), ("log_cases", log_cases),
                     ("table_cases", table_cases)]:
        if only and name not in only:
            continue
        d = fn()
        d["provenance"] = provenance
        with open(os.path.join(GOLDEN, f"{name}.json"), "w") as f:
            json.dump(d, f, separators=(",", ":"))
        print("wrote", name)
    if "cfg5" in only:  # added to the existing configs.json (10^7 blocks: minutes of CPU)
        path = os.path.join(GOLDEN, "configs.json")
        with open(path) as f:
            d = json.load(f)
        new = cfg5()
        if "cfg5" in d:  # regenerated (e.g. to add fields): the pinned values must not move
            for k in ("digest", "crc_last", "crc_first", "sub_digests"):
                assert new[k] == d["cfg5"][k], f"cfg5 {k} changed"
        d["cfg5"] = new
        with open(path, "w") as f:
            json.dump(d, f, indent=1)
        print("cfg5 digest", hex(d["cfg5"]["digest"]), "crc_last", hex(d["cfg5"]["crc_last"]))
    if "cfg2_union" in only:  # added to the existing configs.json
        path = os.path.join(GOLDEN, "configs.json")
        with open(path) as f:
            d = json.load(f)
        d["cfg2_union"] = cfg2_union()
        with open(path, "w") as f:
            json.dump(d, f, indent=1)
        print("cfg2_union", {k: hex(v["digest"]) for k, v in d["cfg2_union"].items() if isinstance(v, dict)})
    if only and "configs" not in only:
        return
    d = configs(not args.no_cfg4)
    try:  # keep cfg5 / cfg2_union made earlier (--only cfg5,cfg2_union)
        with open(os.path.join(GOLDEN, "configs.json")) as f:
            old = json.load(f)
        for k in ("cfg5", "cfg2_union"):
            if k in old:
                d[k] = old[k]
    except (OSError, ValueError):
        pass
    d["provenance"] = provenance
    with open(os.path.join(GOLDEN, "configs.json"), "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps({k: {kk: (hex(vv) if isinstance(vv, int) and kk in ("digest", "crc_last") else vv)
                          for kk, vv in v.items() if kk != "crc_first"}
                      for k, v in d.items() if k.startswith("cfg")}, indent=1))


if __name__ == "__main__":
    main()
