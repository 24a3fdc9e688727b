"""Log-file scenarios for the framing shims (tests/test_framing.py) and their
golden traces (oracle/gen_golden.py -> tests/golden/log_cases.json).

A scenario is data: the records written (payload sizes + a seed; payload
bytes come from the splitmix stream), in one or more append segments (a
writer reopened on a file of the current length, db/log_writer.cc:24-27), then
byte-level mutations, then a read with a checksum flag and an initial offset.
The named scenarios follow the cases of the reference's db/log_test.cc; the
rest are seeded random ones.  Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

B = 32768  # db/log_format.h:27 kBlockSize
H = 7      # db/log_format.h:30 kHeaderSize


def payloads(port, seg: dict) -> list[bytes]:
    seed = seg["seed"]
    return [port.fill(seed + i, 0, n).tobytes() for i, n in enumerate(seg["sizes"])]


def write_image(port, spec: dict, writer) -> bytes:
    """writer(payloads, dest_length) -> the bytes one log::Writer appends."""
    img = b""
    for seg in spec["segments"]:
        img += writer(payloads(port, seg), len(img))
    return img


def mutate(port, img: bytes, muts: list) -> bytes:
    b = bytearray(img)
    for m in muts:
        op = m[0]
        if op == "xor":        # ("xor", pos, value)
            b[m[1]] ^= m[2]
        elif op == "set":      # ("set", pos, byte)
            b[m[1]] = m[2]
        elif op == "truncate":  # ("truncate", drop_bytes)
            del b[len(b) - m[1]:]
        elif op == "fill":     # ("fill", pos, n, byte)
            b[m[1]:m[1] + m[2]] = bytes([m[3]]) * m[2]
        elif op == "append":   # ("append", n, byte)
            b += bytes([m[2]]) * m[1]
        elif op == "fixcrc":   # ("fixcrc", header_pos): re-seal one header as the writer would
            p = m[1]
            n = b[p + 4] | (b[p + 5] << 8)
            crc = port.mask(port.value(bytes(b[p + 6:p + 7 + n])))
            b[p:p + 4] = int(crc).to_bytes(4, "little")
        else:
            raise ValueError(op)
    return bytes(b)


def _seg(sizes, seed):
    return {"sizes": [int(x) for x in sizes], "seed": int(seed)}


def named() -> list[dict]:
    """The db/log_test.cc cases (names follow its TEST()s)."""
    S = []

    def add(name, segs, muts=(), checksum=True, initial_offset=0):
        S.append({"name": name, "segments": segs, "mutations": [list(m) for m in muts],
                  "checksum": checksum, "initial_offset": int(initial_offset)})

    add("Empty", [_seg([], 1)])
    add("ReadWrite", [_seg([3, 3, 0, 4], 2)])
    add("ManyBlocks", [_seg([1 + (i % 6) for i in range(100000)], 3)])
    add("Fragmentation", [_seg([5, 50000, 100000], 4)])
    add("MarginalTrailer", [_seg([B - 2 * H, 0, 3], 5)])
    add("MarginalTrailer2", [_seg([B - 2 * H, 3], 6)])
    add("ShortTrailer", [_seg([B - 2 * H + 4, 0, 3], 7)])
    add("AlignedEof", [_seg([B - 2 * H + 4], 8)])
    add("OpenForAppend", [_seg([5], 9), _seg([5], 10)])
    add("OpenForAppendBlockEdge", [_seg([B - H - 3], 11), _seg([10, 0, 70000], 12)])
    rng = np.random.default_rng(301)
    add("RandomRead", [_seg(np.minimum(rng.integers(0, 1 << rng.integers(0, 17, 500)), 100000), 13)])
    add("BadRecordType", [_seg([3], 14)], [("set", 6, 100), ("fixcrc", 0)])
    add("TruncatedTrailingRecordIsIgnored", [_seg([3], 15)], [("truncate", 4)])
    add("BadLength", [_seg([B - H, 3], 16)], [("xor", 4, 1)])
    add("BadLengthAtEndIsIgnored", [_seg([3], 17)], [("truncate", 1)])
    add("ChecksumMismatch", [_seg([3], 18)], [("xor", 0, 10)])
    add("ChecksumMismatchNoVerify", [_seg([3], 18)], [("xor", 0, 10)], checksum=False)
    add("UnexpectedMiddleType", [_seg([3], 19)], [("set", 6, 3), ("fixcrc", 0)])
    add("UnexpectedLastType", [_seg([3], 20)], [("set", 6, 4), ("fixcrc", 0)])
    add("UnexpectedFullType", [_seg([3, 3], 21)], [("set", 6, 2), ("fixcrc", 0)])
    add("UnexpectedFirstType", [_seg([3, 100000], 22)], [("set", 6, 2), ("fixcrc", 0)])
    add("MissingLastIsIgnored", [_seg([2 * B], 23)], [("truncate", 14)])
    add("PartialLastIsIgnored", [_seg([2 * B], 24)], [("truncate", 1)])
    add("SkipIntoMultiRecord", [_seg([3 * B, 7], 25)], initial_offset=B)
    add("ErrorJoinsRecords", [_seg([B, B, 7], 26)], [("fill", B, B, ord("x"))])
    add("ZeroFilledTail", [_seg([10, 20, 30], 27)], [("append", 40000, 0)])
    add("ZeroRecordMidBlock", [_seg([10, 20, 30], 28)], [("fill", 17, 7, 0)])
    add("TrailingGarbageShortOfHeader", [_seg([10], 29)], [("append", 5, 0x41)])
    # log_test.cc initial-offset family: record sizes of its initial_offset_record_sizes_
    sizes = [10000, 10000, 2 * B - 1000, 1, 13716, B - H]
    probe = sorted({0, 1, 10000, 10007, 10008, 20014, 20015, B - 6, B - 5, B, B + 1, 2 * B - 3, 2 * B,
                    3 * B, 3 * B + 17, 4 * B - 1, 4 * B, 10 * B})
    for off in probe:
        add(f"InitialOffset_{off}", [_seg(sizes, 30)], initial_offset=off)
    return S


def random_cases(count: int, seed: int = 4242) -> list[dict]:
    """Seeded random scenarios: random record sizes, 0-3 mutations, random
    initial offsets and checksum flags."""
    rng = np.random.default_rng(seed)
    S = []
    for c in range(count):
        nseg = 1 if rng.random() < 0.8 else 2
        segs = []
        for _ in range(nseg):
            nrec = int(rng.integers(0, 40))
            mode = rng.random()
            if mode < 0.5:
                sizes = rng.integers(0, 300, nrec)
            elif mode < 0.8:
                sizes = rng.integers(0, 3 * B, nrec)
            else:
                sizes = np.minimum(rng.integers(0, 1 << rng.integers(0, 18, nrec)), 4 * B)
            segs.append(_seg(sizes, int(rng.integers(1, 2**31))))
        # mutation positions are drawn as fractions and resolved against the image later
        muts = []
        for _ in range(int(rng.integers(0, 4))):
            kind = rng.choice(["xor", "set_type", "truncate", "fill0", "len"])
            f = float(rng.random())
            muts.append([str(kind), f, int(rng.integers(1, 256))])
        S.append({"name": f"Random_{c}", "segments": segs, "mutations_rel": muts,
                  "checksum": bool(rng.random() < 0.9),
                  "initial_offset_rel": float(rng.random()) if rng.random() < 0.3 else 0.0})
    return S


def resolve(port, spec: dict, img: bytes) -> tuple[list, int]:
    """Concrete mutations and initial offset for a scenario whose positions
    are relative (random_cases) -- a pure function of the clean image."""
    if "mutations" in spec:
        return spec["mutations"], spec["initial_offset"]
    muts = []
    n = len(img)
    for kind, f, v in spec["mutations_rel"]:
        if n == 0:
            break
        p = min(n - 1, int(f * n))
        if kind == "xor":
            muts.append(["xor", p, v])
        elif kind == "truncate":
            muts.append(["truncate", 1 + p % min(n, 40)])
            n -= 1 + p % min(n, 40)
        elif kind == "fill0":
            muts.append(["fill", p, min(n - p, 1 + v * 7), 0])
        elif kind in ("set_type", "len"):
            # a header-ish position: the start of the block containing p, if a header is there
            h = p - p % B
            if h + H <= n:
                if kind == "set_type":
                    muts.append(["set", h + 6, v % 7])
                    muts.append(["fixcrc", h])
                else:
                    muts.append(["xor", h + 4 + (v & 1), v])
    io = int(spec["initial_offset_rel"] * (len(img) + B))
    return muts, io
