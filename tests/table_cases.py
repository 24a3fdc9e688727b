"""SSTable scenarios for the whole-table verify shim (nvl_sstable_verify_table,
tests/test_table_verify.py) and their golden traces (oracle/gen_golden.py ->
tests/golden/table_cases.json).

A scenario is data: a seed and block counts from which `build` writes a
table image in the reference's on-disk format -- data blocks in the
BlockBuilder layout (prefix-compressed entries, a restart every 16 keys,
table/block_builder.cc), an optional filter-like meta block, the metaindex
block, the index block (restart interval 1, one BlockHandle per data block,
table/table_builder.cc:200-250), every block followed by type | Mask(CRC)
(table_builder.cc:175-193), and the 48-byte footer (table/format.cc:32-41) --
then an index "mode" that writes a malformed but correctly sealed index, then
byte-level mutations.  The named scenarios cover each Table::Open / ReadBlock
/ Block::Iter outcome; the rest are seeded random ones.  Block CRCs come from
the oracle port (pinned against the reference, tests/test_oracle.py).
Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

MAGIC = 0xDB4775248B80FB57  # table/format.h:77
FOOTER = 48                 # Footer::kEncodedLength


def varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def handle(off: int, size: int) -> bytes:
    return varint(off) + varint(size)


def _varint_handle(v: bytes) -> tuple[int, int]:
    """handle() decoded back -> (offset, size)."""
    out, shift, acc = [], 0, 0
    for c in v:
        acc |= (c & 127) << shift
        shift += 7
        if c < 128:
            out.append(acc)
            acc, shift = 0, 0
    return out[0], out[1]


def varint32_wrapped(x: int) -> bytes:
    """x < 2^28 as a 5-byte varint whose last byte carries bit 32: the
    reference's GetVarint32PtrFallback (util/coding.cc:112-129) accumulates
    into a uint32_t and drops it, so it still decodes x."""
    return bytes([(x & 127) | 128, ((x >> 7) & 127) | 128, ((x >> 14) & 127) | 128, ((x >> 21) & 127) | 128,
                  ((x >> 28) & 15) | 0x10])


def block(entries: list[tuple[bytes, bytes]], restart_interval: int, force_varint: bool = False,
          wrap32: bool = False) -> bytes:
    """BlockBuilder layout (table/block_builder.cc): shared | non_shared |
    value_len (varint32) | key delta | value, then the restart array."""
    out = bytearray()
    restarts = [0]
    last = b""
    for i, (k, v) in enumerate(entries):
        if i and i % restart_interval == 0:
            restarts.append(len(out))
            last = b""
        shared = 0
        while shared < min(len(last), len(k)) and last[shared] == k[shared]:
            shared += 1
        if force_varint:  # multi-byte encodings of small values (still valid varints)
            out += bytes([shared | 128, 0]) + bytes([(len(k) - shared) | 128, 0]) + bytes([len(v) | 128, 0])
        elif wrap32:  # 5-byte encodings with bit 32 set (truncated by the reference's decoder)
            out += varint32_wrapped(shared) + varint32_wrapped(len(k) - shared) + varint32_wrapped(len(v))
        else:
            out += varint(shared) + varint(len(k) - shared) + varint(len(v))
        out += k[shared:] + v
        last = k
    for r in restarts:
        out += r.to_bytes(4, "little")
    out += len(restarts).to_bytes(4, "little")
    return bytes(out)


class _Writer:
    def __init__(self, port):
        self.port = port
        self.img = bytearray()

    def raw(self, contents: bytes, btype: int = 0) -> tuple[int, int]:
        off = len(self.img)
        self.img += contents + bytes([btype])
        self.img += int(self.port.mask(self.port.value(contents + bytes([btype])))).to_bytes(4, "little")
        return off, len(contents)


def build(port, spec: dict) -> tuple[bytes, dict]:
    """-> (image, layout): layout holds the handles the writer placed."""
    rng = np.random.default_rng(spec["seed"])
    w = _Writer(port)
    data = []
    key = 0
    for b in range(spec["nblocks"]):
        n = int(rng.integers(0 if spec.get("empty_blocks") else 1, 40))
        ents = []
        for _ in range(n):
            key += int(rng.integers(1, 1000))
            v = port.fill(spec["seed"] * 7919 + key, 0, int(rng.integers(0, 200))).tobytes()
            ents.append((b"user-key-%012d" % key, v))
        data.append((w.raw(block(ents, 16)), b"user-key-%012d" % key))
    meta = []
    for m in range(spec.get("nmeta", 1)):
        filt = port.fill(spec["seed"] * 31 + m, 0, int(rng.integers(0, 600))).tobytes()
        meta.append((b"filter.leveldb.BuiltinBloomFilter%d" % (m + 2), w.raw(filt)))
    ments = [(k, handle(*h)) for k, h in meta]
    if spec.get("meta_mode") == "bad_handle" and ments:  # a metaindex value that is not a BlockHandle
        ments[0] = (ments[0][0], b"\xff")
    meta_h = w.raw(block(ments, 16))
    mode = spec.get("index_mode", "")
    ents = [(k, handle(*h)) for h, k in data]
    if mode == "bad_handle" and ents:      # a value that is not a BlockHandle (table.cc:160-165)
        i = int(rng.integers(0, len(ents)))
        ents[i] = (ents[i][0], b"\xff")
    if mode == "past_end" and ents:        # a handle beyond the file end
        i = int(rng.integers(0, len(ents)))
        ents[i] = (ents[i][0], handle(len(w.img) + 10000, 100))
    if mode == "big_size" and ents:        # a handle whose size exceeds the file
        i = int(rng.integers(0, len(ents)))
        ents[i] = (ents[i][0], handle(data[i][0][0], 1 << 40))
    if mode == "overlap" and len(ents) > 1:  # a handle straddling two blocks (reads, checksum mismatch)
        ents[0] = (ents[0][0], handle(data[0][0][0] + 1, data[0][0][1]))
    idx = block(ents, 1, force_varint=(mode == "varint"), wrap32=(mode == "varint32_wrap"))
    if mode == "bad_entry" and ents:       # shared > previous key length -> "bad entry in block"
        cut = int(rng.integers(0, len(ents)))
        body, starts = b"", []
        for k, v in ents[:cut]:
            starts.append(len(body))
            body += varint(0) + varint(len(k)) + varint(len(v)) + k + v
        starts.append(len(body))
        k, v = ents[cut]
        body += varint(200) + varint(len(k)) + varint(len(v)) + k + v
        idx = body + b"".join(x.to_bytes(4, "little") for x in starts) + len(starts).to_bytes(4, "little")
    if mode == "overrun" and ents:         # an entry running past the restart array
        idx = varint(0) + varint(90) + varint(90) + b"x" * 10 + (0).to_bytes(4, "little") + (1).to_bytes(4, "little")
    if mode == "bad_restarts":             # num_restarts larger than the block -> "bad block contents"
        idx = idx[:-4] + (1 << 20).to_bytes(4, "little")
    if mode == "tiny":                     # < 4 bytes
        idx = b"\x01"
    if mode == "empty":                    # zero restarts: an empty index
        idx = (0).to_bytes(4, "little")
    if mode == "restart0_past":            # restart point 0 beyond the entries: no entries
        idx = idx[:-8] + (len(idx) + 50).to_bytes(4, "little") + idx[-4:] if len(ents) == 1 else idx
    index_h = w.raw(idx, 1 if mode == "compressed" else 0)
    foot = handle(*meta_h) + handle(*index_h)
    foot += bytes(40 - len(foot)) + MAGIC.to_bytes(8, "little")
    if mode == "bad_footer":
        foot = b"\xff" * 40 + foot[40:]
    w.img += foot
    img = bytes(w.img)
    layout = {"data": [h for h, _ in data], "meta": [h for _, h in meta], "metaindex": meta_h, "index": index_h}
    return mutate(port, img, spec.get("muts", []), layout), layout


def mutate(port, img: bytes, muts: list, layout: dict) -> bytes:
    b = bytearray(img)

    def reseal(off, n):
        b[off + n + 1:off + n + 5] = int(port.mask(port.value(bytes(b[off:off + n + 1])))).to_bytes(4, "little")

    for m in muts:
        op = m[0]
        if op == "flip":        # ("flip", role, k, pos_frac, bit): a content byte -> checksum mismatch
            off, n = _pick(layout, m[1], m[2])
            if n:
                b[off + int(m[3] * n) % n] ^= 1 << m[4]
        elif op == "type":      # ("type", role, k, t): type byte t, resealed
            off, n = _pick(layout, m[1], m[2])
            b[off + n] = m[3]
            reseal(off, n)
        elif op == "crc":       # ("crc", role, k, byte): a stored CRC byte
            off, n = _pick(layout, m[1], m[2])
            b[off + n + 1 + m[3]] ^= 0x21
        elif op == "magic":
            b[-1] ^= 0x01
        elif op == "truncate":  # ("truncate", n_bytes)
            del b[len(b) - m[1]:]
        else:
            raise ValueError(op)
    return bytes(b)


def _pick(layout, role, k):
    if role == "data":
        return layout["data"][k % len(layout["data"])]
    if role == "meta":
        return layout["meta"][k % len(layout["meta"])]
    return layout[role]


def named() -> list[dict]:
    c = []

    def add(name, **kw):
        spec = {"name": name, "seed": 100 + len(c), "nblocks": 6, "nmeta": 1}
        spec.update(kw)
        c.append(spec)

    add("clean")
    add("clean_many", nblocks=300, nmeta=2)
    add("no_data_blocks", nblocks=0)
    add("no_meta", nmeta=0)
    add("empty_data_blocks", empty_blocks=True, nblocks=10)
    add("data_checksum", muts=[("flip", "data", 2, 0.5, 3)])
    add("data_bad_type", muts=[("type", "data", 1, 7)])
    add("data_type1", muts=[("type", "data", 3, 1)])
    add("data_crc_byte", muts=[("crc", "data", 0, 2)])
    add("meta_checksum", muts=[("flip", "meta", 0, 0.3, 1)])
    add("metaindex_checksum", muts=[("flip", "metaindex", 0, 0.5, 0)])
    add("metaindex_bad_type", muts=[("type", "metaindex", 0, 9)])
    add("index_checksum", muts=[("flip", "index", 0, 0.5, 6)])
    add("index_bad_type", muts=[("type", "index", 0, 200)])
    add("bad_magic", muts=[("magic",)])
    add("too_short", muts=[("truncate", 10 ** 9)])
    add("truncated_tail", muts=[("truncate", 3)])
    add("bad_footer", index_mode="bad_footer")
    add("bad_handle", index_mode="bad_handle")
    add("past_end", index_mode="past_end")
    add("big_size", index_mode="big_size")
    add("overlap", index_mode="overlap")
    add("varint_entries", index_mode="varint")
    add("bad_entry", index_mode="bad_entry", nblocks=9)
    add("overrun", index_mode="overrun")
    add("bad_restarts", index_mode="bad_restarts")
    add("tiny_index", index_mode="tiny")
    add("empty_index", index_mode="empty")
    add("compressed_index", index_mode="compressed")
    add("restart0_past", index_mode="restart0_past", nblocks=1)
    add("varint32_wrap", index_mode="varint32_wrap", nblocks=5)
    add("meta_bad_handle", meta_mode="bad_handle", nmeta=2)
    return c


def random_cases(count: int, seed: int = 777) -> list[dict]:
    rng = np.random.default_rng(seed)
    modes = ["", "", "", "", "bad_handle", "past_end", "big_size", "overlap", "varint", "bad_entry"]
    out = []
    for i in range(count):
        nb = int(rng.integers(0, 40))
        nmeta = int(rng.integers(0, 3))
        muts = []
        for _ in range(int(rng.integers(0, 5))):
            role = str(rng.choice(["data", "data", "data", "meta", "metaindex", "index"]))
            if (role == "data" and nb == 0) or (role == "meta" and nmeta == 0):
                continue
            what = int(rng.integers(0, 3))
            k = int(rng.integers(0, 1000))
            if what == 0:
                muts.append(("flip", role, k, float(rng.random()), int(rng.integers(0, 8))))
            elif what == 1 and role in ("data", "meta"):
                muts.append(("type", role, k, int(rng.choice([1, 2, 3, 255]))))
            else:
                muts.append(("crc", role, k, int(rng.integers(0, 4))))
        out.append({"name": f"random_{i}", "seed": 5000 + i, "nblocks": nb, "nmeta": nmeta,
                    "index_mode": str(rng.choice(modes)), "muts": muts})
    return out


# ---- reference trace -> expected shim output ------------------------------

_VERDICT = {"OK": 0, "Corruption: truncated block read": 1, "Corruption: block checksum mismatch": 2,
            "Corruption: bad block type": 3, "Corruption: bad block handle": 4,
            "Corruption: corrupted compressed block contents": 0}  # type-1 blocks: decompression is out of scope
_TABLE = {"Corruption: file is too short to be an sstable": 1, "Corruption: not an sstable (bad magic number)": 2,
          "Corruption: bad block handle": 3}


def expected(trace: str) -> tuple[int, list[tuple[int, int, int, int]]]:
    """ref_table_scan trace -> (NVL_TABLE_*, [(offset, size, role, verdict)]) in
    the shim's order (index, metaindex, meta blocks, data blocks)."""
    by_role: dict[int, list] = {0: [], 1: [], 2: [], 3: []}
    status = 0
    for line in trace.splitlines():
        if line.startswith("T "):
            return _TABLE[line[2:]], []
        if line.startswith("S 0 "):
            status = {"Corruption: bad entry in block": 6, "Corruption: bad block contents": 5}[line[4:]]
        elif line.startswith("B "):
            _, role, off, size, msg = line.split(" ", 4)
            v = 1 if msg.startswith("IO error") else _VERDICT[msg]
            by_role[int(role)].append((int(off), int(size), int(role), v))
    idx = by_role[0][0]
    if trace.startswith("B 0 ") and trace.split("\n", 1)[0].endswith("corrupted compressed block contents"):
        return 7, [idx]  # the index block is stored compressed: not parsed by the shim
    if idx[3] != 0:
        return 4, [idx]
    return status, by_role[0] + by_role[1] + by_role[2] + by_role[3]
