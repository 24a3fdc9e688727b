"""Pure-Python model of the HIP engine's algorithm (test infrastructure).

Mirrors nvlevelz_amd/csrc/crc32c_*.hip / crc32c_dev*.h step for step -- end-aligned
4096-byte chunks, 64 lanes x 64-byte pieces, leading-zero masking and ~init
injection, per-lane slice-by-4, the 6-level shift-operator butterfly, the
per-wave contiguous chunk ranges with shift4096 accumulation, the per-wave
head/tail records and the fix-up fold -- so the decomposition can be checked
against the oracle on the CPU, at small sizes, before any GPU run.  It also
holds the GF(2) helpers restated from crc32c_math.h.
"""
from __future__ import annotations

POLY = 0x82F63B78
ONE = 0x80000000
CHUNK = 4096


def gf_mul(a: int, b: int) -> int:
    p = 0
    for i in range(32):
        if a & (ONE >> i):
            p ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return p


X2N = []
_p = ONE >> 1
for _k in range(64):
    X2N.append(_p)
    _p = gf_mul(_p, _p)


def xpow8(n: int) -> int:
    p, k = ONE, 3
    while n:
        if n & 1:
            p = gf_mul(X2N[k], p)
        n >>= 1
        k += 1
    return p


def shift(v: int, nbytes: int) -> int:
    return gf_mul(xpow8(nbytes), v)


def _t0(b: int) -> int:
    c = b
    for _ in range(8):
        c = (c >> 1) ^ (POLY if c & 1 else 0)
    return c


T = [[_t0(b) for b in range(256)]]
for _k in range(1, 4):
    T.append([(T[_k - 1][b] >> 8) ^ T[0][T[_k - 1][b] & 0xFF] for b in range(256)])


def shift_op(dist: int):
    m = xpow8(dist)
    return [[gf_mul(m, b << (8 * j)) for b in range(256)] for j in range(4)]


COMB = [shift_op(64 << lev) for lev in range(6)]
SH4096 = shift_op(4096)


def slice4(x: int) -> int:
    return T[3][x & 0xFF] ^ T[2][(x >> 8) & 0xFF] ^ T[1][(x >> 16) & 0xFF] ^ T[0][x >> 24]


def apply_op(op, v: int) -> int:
    return op[0][v & 0xFF] ^ op[1][(v >> 8) & 0xFF] ^ op[2][(v >> 16) & 0xFF] ^ op[3][v >> 24]


def raw_bytes(state: int, data: bytes) -> int:
    for b in data:
        state = T[0][(state ^ b) & 0xFF] ^ (state >> 8)
    return state


# ---- the wave algorithm ----------------------------------------------------

def wave_fold(g):
    """Butterfly over 64 lane values exactly as fold_level<0..5>."""
    g = list(g)
    for lev in range(6):
        pt = [g[l ^ (1 << lev)] for l in range(64)]
        new = [0] * 64
        # every lane computes the same thing within its group; model per lane
        for l in range(64):
            hi = (l >> lev) & 1
            left = pt[l] if hi else g[l]
            right = g[l] if hi else pt[l]
            new[l] = apply_op(COMB[lev], left) ^ right
        g = new
    assert len(set(g)) == 1
    return g[0]


OVER = 0  # overhang (round-1 knob, removed from the kernels): a first chunk of up to 4096 + OVER bytes is ONE pass


def chunks_of(L: int) -> int:
    """Chunks of a buffer of L bytes (crc32c_dev.h chunks_for): END-aligned
    4096-byte chunks (with an overhang, a first chunk of 4097..4096+OVER bytes
    is not split)."""
    return 1 if L <= CHUNK + OVER else (L - OVER + CHUNK - 1) // CHUNK


def _mask_inject(words, rel: int, s: int):
    """Zero the bytes of a piece before the buffer start (rel = bytes of the
    piece before it) and XOR ~init (s) into the 4 bytes at the start."""
    rel = max(-8, min(72, rel))
    out = []
    for k, w in enumerate(words):
        sh = rel - 4 * k
        keep = 0xFFFFFFFF if sh <= 0 else (0 if sh >= 4 else (0xFFFFFFFF << (8 * sh)) & 0xFFFFFFFF)
        inj = 0
        if 0 <= sh < 4:
            inj = (s << (8 * sh)) & 0xFFFFFFFF
        elif -4 < sh < 0:
            inj = s >> (-8 * sh)
        out.append((w & keep) ^ inj)
    return out


def group_fold(g, nlev: int):
    """The first nlev butterfly levels over a lane group (fold_level<0..nlev-1>)."""
    g = list(g)
    for lev in range(nlev):
        new = []
        for l in range(len(g)):
            pt = g[l ^ (1 << lev)]
            hi = (l >> lev) & 1
            left, right = (pt, g[l]) if hi else (g[l], pt)
            new.append(apply_op(COMB[lev], left) ^ right)
        g = new
    assert len(set(g)) == 1
    return g[0]


def head_class(hl: int) -> int:
    """Lanes per head (crc32c_dev_heads.h run_heads): 64-byte pieces, P = 1, 4, 16, 64."""
    return 1 if hl <= 64 else 4 if hl <= 256 else 16 if hl <= 1024 else 64


def head_raw(mem: bytes, p: int, L: int, J: int, s: int) -> int:
    """Raw register of buffer [p, p+L)'s head (partial first chunk, 1..4095
    bytes) the way head_load / head_raw run it: a group of P lanes, lane k's
    piece [ce - 64P + 64k, +64) read as four 16-byte slots from the 4-byte
    aligned A4 at or below it plus the dword at A4 + 64; a slot wholly below
    p's granule g is not loaded, the one straddling g is loaded from g."""
    hl = L - CHUNK * (J - 1)
    assert 4 <= hl < CHUNK or (J > 1 and 1 + OVER <= hl < CHUNK)
    ce = p + hl
    g = p & ~15
    P = head_class(hl)

    def load(a: int, n: int) -> bytes:
        # fault safety: only 16-B granules holding bytes of [p, ce)
        assert (a & ~15) >= g and ((a + n - 1) & ~15) <= ((ce - 1) & ~15), (a, n, p, ce)
        return mem[a:a + n]

    lanes = []
    for k in range(P):
        ps = ce - 64 * P + 64 * k
        A4 = ps & ~3
        d = bytearray(68)
        for j in range(4):
            a = A4 + 16 * j
            if a + 16 <= g:
                continue
            if a < g:
                d[16 * j + (g - a):16 * j + 16] = load(g, 16)[:16 - (g - a)]
            else:
                d[16 * j:16 * j + 16] = load(a, 16)
        if ps & 3 and A4 + 68 > g:
            d[64:68] = load(A4 + 64, 4)
        b = ps & 3
        words = [int.from_bytes(d[b + 4 * q:b + 4 * q + 4], "little") for q in range(16)]
        words = _mask_inject(words, p - ps, s)
        crc = 0
        for w in words:
            crc = slice4(crc ^ w)
        lanes.append(crc)
    return group_fold(lanes, P.bit_length() - 1)


def long_head(p: int, hl: int) -> bool:
    """crc32c_dev_heads.h run_heads: a head of 1025..4095 bytes runs as a whole
    chunk (long_heads) unless the buffer starts in the first 16 bytes of a
    4 KiB page."""
    return 1024 < hl < CHUNK and ((p >> 4) & 255) != 0


def long_head_raw(mem: bytes, p: int, L: int, J: int, s: int) -> int:
    """Raw register of a long head the way long_heads runs it
    (load_general / realign_general with hd): the chunk [ce - 4096, ce) loaded
    as 256 16-byte row slots from the 4-byte aligned A4 at or below its start
    plus the dword holding byte ce - 1; a slot wholly below p's granule g is
    loaded from g (garbage), the one straddling g reads up to 12 bytes below
    g, which must lie in g's 4 KiB page; bytes before p zeroed and ~init
    injected at p (head_fix)."""
    hl = L - CHUNK * (J - 1)
    assert long_head(p, hl)
    ce = p + hl
    cs = ce - CHUNK
    g = p & ~15
    A4 = cs & ~3
    r = cs & 3

    def load(a: int, n: int) -> bytes:
        # fault safety: granules up to the one holding ce - 1; below g only
        # inside g's page
        assert ((a + n - 1) & ~15) <= ((ce - 1) & ~15), (a, n, p, ce)
        assert (a & ~15) >= g or (a >> 12) == (g >> 12), (a, n, p, g)
        return mem[a:a + n]

    data = bytearray(CHUNK + 4)
    for k in range(CHUNK // 16):
        a = A4 + 16 * k
        data[16 * k:16 * k + 16] = load(g if a + 16 <= g else a, 16)
    data[CHUNK:CHUNK + 4] = load((ce - 1) & ~3, 4)
    piece = bytearray(data[r:r + CHUNK])  # bytes [cs, ce), garbage before p
    rel = p - cs
    piece[:rel] = bytes(rel)
    for q in range(4):
        piece[rel + q] ^= (s >> (8 * q)) & 0xFF
    lanes = []
    for lane in range(64):
        crc = 0
        for k in range(16):
            crc = slice4(crc ^ int.from_bytes(piece[64 * lane + 4 * k:64 * lane + 4 * k + 4], "little"))
        lanes.append(crc)
    return wave_fold(lanes)


def masked_pass_raw(mem: bytes, p: int, L: int, s: int) -> int:
    """Raw register of a one-chunk buffer of 1025..4095 bytes as a kMasked
    scheduler-A pass (crc32c_fixed_kernel<kGeneral>: load_general with hd,
    page_head_words, realign_general with hd), at ANY start: the row slot
    straddling p's granule g reads up to 12 bytes below g -- unless g is a
    page's first granule, where it is loaded from g and its words are moved up
    by (g - x) / 4 dwords.  Fault safety: below g only inside g's page."""
    assert 1025 <= L < CHUNK
    ce = p + L
    cs = ce - CHUNK
    g = p & ~15
    A4 = cs & ~3
    r = cs & 3
    gl = g - 15 if g & 4095 else g

    def load(a: int, n: int) -> bytes:
        assert ((a + n - 1) & ~15) <= ((ce - 1) & ~15), (a, n, p, ce)
        assert (a & ~15) >= g or (a >> 12) == (g >> 12), (a, n, p, g)
        return mem[a:a + n]

    data = bytearray(CHUNK + 4)
    for k in range(CHUNK // 16):
        x = A4 + 16 * k
        slot = bytearray(load(g if x < gl else x, 16))
        if not g & 4095 and x < g < x + 16:  # page_head_words
            q = (g - x) // 4
            slot = bytearray(4 * q) + slot[:16 - 4 * q]
        data[16 * k:16 * k + 16] = slot
    data[CHUNK:CHUNK + 4] = load((ce - 1) & ~3, 4)
    piece = bytearray(data[r:r + CHUNK])
    rel = p - cs
    piece[:rel] = bytes(rel)
    for q in range(4):
        piece[rel + q] ^= (s >> (8 * q)) & 0xFF
    lanes = []
    for lane in range(64):
        crc = 0
        for k in range(16):
            crc = slice4(crc ^ int.from_bytes(piece[64 * lane + 4 * k:64 * lane + 4 * k + 4], "little"))
        lanes.append(crc)
    return wave_fold(lanes)


def chunk_raw(mem: bytes, p: int, L: int, J: int, c: int, s: int) -> int:
    """Raw register of chunk c of buffer [p, p+L) with ~init = s injected,
    computed the way load_chunk<kGeneral> / build_words<kGeneral> do it (a
    partial first chunk: the head kernel, long_head_raw or head_raw)."""
    e = p + L
    if c == 0 and e - CHUNK * (J - 1) - CHUNK < p:
        if L >= 4 and long_head(p, L - CHUNK * (J - 1)):
            return long_head_raw(mem, p, L, J, s)
        return head_raw(mem, p, L, J, s)
    ce = e - CHUNK * (J - 1 - c)
    cs = ce - CHUNK
    r = ce & 3
    A4 = cs - r  # every chunk is loaded from the 4-byte aligned address below its start
    g = p & ~15

    def load(a: int, n: int) -> bytes:
        # fault safety: only 16-B granules that hold buffer bytes are touched
        assert (a & ~15) >= g and ((a + n - 1) & ~15) <= ((e - 1) & ~15), (a, n, p, e)
        return mem[a:a + n]

    slots = bytearray(CHUNK + 4)
    for k in range(CHUNK // 16):
        slots[16 * k:16 * k + 16] = load(A4 + 16 * k, 16)
    if r:  # lane 63's 16-byte edge load ending at A4 + 4100
        edge = load(A4 + CHUNK - 12, 16)
        slots[CHUNK:CHUNK + 4] = edge[12:16]
    lanes = []
    for lane in range(64):
        piece = slots[r + 64 * lane:r + 64 * lane + 64]  # bytes [cs + 64 lane, +64)
        words = [int.from_bytes(piece[4 * k:4 * k + 4], "little") for k in range(16)]
        if lane == 0 and p <= cs < p + 4:
            words[0] ^= s >> (8 * (cs - p))  # ~init, or what a 1..3-byte head / the overhang leaves of it
        crc = 0
        for w in words:
            crc = slice4(crc ^ w)
        lanes.append(crc)
    raw = wave_fold(lanes)
    if c == 0 and cs > p:  # overhang: bytes [p, cs) as a 16-byte piece ending at cs
        o = cs - p
        assert 1 <= o <= OVER
        r2 = cs & 3
        B4 = cs - 16 - r2  # = A4 - 16
        dw = bytearray(20)
        ea = max(B4, g)  # lane 0's 16-byte edge load, clamped up to g
        edge = load(ea, 16)
        dw[ea - B4:16] = edge[:16 - (ea - B4)]
        dw[16:20] = load(B4 + 16, 4)  # lane 0's first loaded dword (A4)
        words = [int.from_bytes(dw[r2 + 4 * k:r2 + 4 * k + 4], "little") for k in range(4)]
        words = _mask_inject(words, p - (cs - 16), s)
        crc = 0
        for w in words:
            crc = slice4(crc ^ w)
        raw ^= apply_op(SH4096, crc)
    return raw


def batch(mem: bytes, bufs, inits, nwaves: int):
    """bufs: list of (p, L).  Returns final CRCs via waves + records + fix-up.
    Records hold NORMALIZED portions: the portion's raw shifted to the end of
    its buffer (4096 * chunks after it), so the fix-up only XORs."""
    n = len(bufs)
    J = [chunks_of(L) for (_, L) in bufs]
    cs = [0]
    for j in J:
        cs.append(cs[-1] + j)
    Ttot = cs[-1]
    out = [None] * n
    recs = []
    NOBUF = -1
    for w in range(nwaves):
        t0, t1 = Ttot * w // nwaves, Ttot * (w + 1) // nwaves
        head, tail = (NOBUF, 0, False), (NOBUF, 0, False)
        if t0 < t1:
            i = max(k for k in range(n) if cs[k] <= t0)
            c = t0 - cs[i]
            from_zero = c == 0
            acc = cnt = 0
            for t in range(t0, t1):
                p, L = bufs[i]
                s = (~inits[i]) & 0xFFFFFFFF
                if L < 4:
                    out[i] = (~raw_bytes(s, mem[p:p + L])) & 0xFFFFFFFF
                    cnt, from_zero = 0, True
                else:
                    raw = chunk_raw(mem, p, L, J[i], c, s)
                    acc = (apply_op(SH4096, acc) ^ raw) if cnt else raw
                    cnt += 1
                    if c + 1 == J[i]:
                        if from_zero:
                            out[i] = (~acc) & 0xFFFFFFFF
                        else:
                            head = (i, acc, True)  # ends the buffer: already normalized
                        cnt, from_zero = 0, True
                    elif t + 1 == t1:  # the unit ends inside buffer i, after its chunk c
                        norm = shift(acc, CHUNK * (J[i] - 1 - c))
                        if from_zero:
                            tail = (i, norm, False)
                        else:
                            head = (i, norm, False)
                if c + 1 == J[i]:
                    i, c = i + 1, 0
                else:
                    c += 1
        recs.append((head, tail))
    # fix-up: XOR of the normalized portions
    for w in range(nwaves):
        h = recs[w][0]
        if h[0] == NOBUF or not h[2]:
            continue
        total = h[1]
        for x in range(w - 1, -1, -1):
            hx, tx = recs[x]
            if hx[0] == h[0]:  # middle portion
                total ^= hx[1]
                continue
            if tx[0] == h[0]:  # first portion
                total ^= tx[1]
                break
            assert hx[0] == NOBUF and tx[0] == NOBUF  # empty-range wave
        else:
            raise AssertionError("first portion not found")
        out[h[0]] = (~total) & 0xFFFFFFFF
    return out


# ---- region path (nvl_crc32c_region_dev) -----------------------------------
# A batch whose buffers lie in ONE region is checksummed over the region's
# page-aligned 4 KiB chunks (crc32c_region_kernel) -- independent of where the
# buffers start -- and each buffer is then derived from chunk-level values
# (crc32c_region_fold_kernel).  Positions are relative to the grid origin
# O = region & ~4095; chunk c covers [4096c, 4096c + 4096).

REGION_DIRECT = 64  # buffers shorter than this are checksummed whole by the fold kernel


def piece_raws(chunk: bytes):
    return [raw_bytes(0, chunk[64 * l:64 * l + 64]) for l in range(64)]


def masked_fold(lane_raws, L: int) -> int:
    """Qe(L): the butterfly over the lanes below L (the others zeroed) -- the
    chunk bytes [0, 64L) zero-extended to the chunk end."""
    return wave_fold([v if l < L else 0 for l, v in enumerate(lane_raws)])


def nibble_table(n: int, v: int, j: int) -> int:
    """The region kernel's LDS nibble tables: T[n][v][j] = shift(v << 4n, 64(63 - j))."""
    return shift(v << (4 * n), 64 * (63 - j))


def lane_scan(lane_raws):
    """crc32c_region_kernel's chunk_scan: each lane moves its piece raw to the
    chunk end through its nibble-table column (lane 63: identity), then an
    inclusive XOR scan over lanes.  Returns (chunk raw, exclusive prefixes):
    pre[L] = Qe(L) = masked_fold(lane_raws, L)."""
    t = []
    for j, v in enumerate(lane_raws):
        if j == 63:
            t.append(v)
            continue
        acc = 0
        for n in range(8):
            acc ^= nibble_table(n, (v >> (4 * n)) & 15, j)
        t.append(acc)
    inc, acc = [], 0
    for x in t:
        acc ^= x
        inc.append(acc)
    return inc[63], [i ^ x for i, x in zip(inc, t)]


def region_events(s: int, e: int, L: int):
    """The (chunk, in-chunk offset) events a buffer [s, e) leaves for the
    chunk kernel: its start unless on a chunk boundary, its end unless on one."""
    ev = []
    if L < REGION_DIRECT:
        return ev
    if s & 4095:
        ev.append(("s", s >> 12, s & 4095))
    if e & 4095:
        ev.append(("e", (e - 1) >> 12, e - ((e - 1) >> 12 << 12)))
    return ev


def piece_prefix_raw(mem: bytes, p: int) -> int:
    """R(p) = raw(0, bytes [p & ~63, p)): what the fold kernel re-reads."""
    return raw_bytes(0, mem[p & ~63:p])


def region_fold(mem: bytes, raws, qe, s: int, L: int, init: int) -> int:
    """Extend(init, mem[s:s+L]) from the chunk raws and the events' Qe, as
    crc32c_region_fold_kernel computes it (xp8[d] = x^(8d), xm8[d] = x^(-8d))."""
    if L < REGION_DIRECT:
        return (~raw_bytes((~init) & 0xFFFFFFFF, mem[s:s + L])) & 0xFFFFFFFF
    e = s + L
    c0, os_ = s >> 12, s & 4095
    c1, oe = (e - 1) >> 12, e - ((e - 1) >> 12 << 12)
    ninit = (~init) & 0xFFFFFFFF
    qs = qe[("s", c0, os_)] if os_ else 0
    rs = piece_prefix_raw(mem, s) if os_ else 0
    # Ze'(s): bytes [cs0, s) at the chunk end, plus ~init injected at s
    zs = qs ^ shift(rs ^ ninit, 4096 - os_)
    if c0 == c1:
        acc = zs
    else:
        acc = raws[c0] ^ zs
        for c in range(c0 + 1, c1):
            acc = apply_op(SH4096, acc) ^ raws[c]
        acc = apply_op(SH4096, acc)
    if oe == 4096:
        v = acc ^ raws[c1]
    else:
        # unshift by 4096 - oe: multiply by x^(-8(4096-oe)), here as a check
        d = 4096 - oe
        v = unshift(acc ^ qe[("e", c1, oe)], d) ^ piece_prefix_raw(mem, e)
    return (~v) & 0xFFFFFFFF


def region_fold_direct(mem: bytes, raws, qe, s: int, L: int, init: int) -> int:
    """The region kernel's fold as it computes a buffer spanning at most two
    chunks, one formula for both (no divergence in a wave that holds both):
    the data terms at chunk c1's end -- Qe(s) directly (one chunk) or
    shift4096(Qe(s) ^ raw c0) (two) -- unshifted to e, plus T x^(8L) and
    R(e): two independent multiplies.  Longer buffers: region_fold."""
    if L < REGION_DIRECT:
        return (~raw_bytes((~init) & 0xFFFFFFFF, mem[s:s + L])) & 0xFFFFFFFF
    e = s + L
    c0, os_ = s >> 12, s & 4095
    c1, oe = (e - 1) >> 12, e - ((e - 1) >> 12 << 12)
    if c1 > c0 + 1:
        return region_fold_steps(mem, raws, qe, s, L, init)
    ninit = (~init) & 0xFFFFFFFF
    qs = qe[("s", c0, os_)] if os_ else 0
    T = (piece_prefix_raw(mem, s) if os_ else 0) ^ ninit
    ze = raws[c1] if oe == 4096 else qe[("e", c1, oe)]
    re = 0 if oe == 4096 else piece_prefix_raw(mem, e)
    back = lambda v: unshift(v, 4096 - oe)  # x^(-8(4096 - oe))
    X = apply_op(SH4096, qs ^ raws[c0]) if c1 == c0 + 1 else qs
    v = back(X ^ ze) ^ shift(T, L) ^ re
    return (~v) & 0xFFFFFFFF


SHC = [shift_op(4096 * d) for d in (1, 2, 3, 4)]  # the fold's chunk shifts (blob shc, LDS kRShcOff)


def region_fold_steps(mem: bytes, raws, qe, s: int, L: int, init: int) -> int:
    """The region kernel's fold of a buffer over three or more chunks
    (fold_out): X = Qe(s) ^ raw c0 at chunk c0's end, then up to four chunks
    per step -- acc at chunk c + k's end = shift(acc, 4096 k) ^ the raws of
    chunks c + 1 .. c + k below c1, each shifted by its distance to c + k --
    unshifted from c1's end, and T = R(s) ^ ~init moved straight to e by
    x^(8L); the same value as region_fold's chunk-by-chunk chain."""
    e = s + L
    c0, os_ = s >> 12, s & 4095
    c1, oe = (e - 1) >> 12, e - ((e - 1) >> 12 << 12)
    assert c1 >= c0 + 2
    ninit = (~init) & 0xFFFFFFFF
    qs = qe[("s", c0, os_)] if os_ else 0
    T = (piece_prefix_raw(mem, s) if os_ else 0) ^ ninit
    acc = qs ^ raws[c0]
    c = c0
    while c < c1:
        k = min(c1 - c, 4)
        x = apply_op(SHC[k - 1], acc)
        for j in range(1, 5):
            rj = raws[c + j] if c + j < c1 else 0
            x ^= apply_op(SHC[k - j - 1], rj) if j < k else rj
        acc, c = x, c + k
    ze = raws[c1] if oe == 4096 else qe[("e", c1, oe)]
    re = 0 if oe == 4096 else piece_prefix_raw(mem, e)
    v = unshift(acc ^ ze, 4096 - oe) ^ shift(T, L) ^ re
    return (~v) & 0xFFFFFFFF


def _xinv(v: int) -> int:
    """v * x^-1 mod P (reflected): the inverse of one zero-bit feed."""
    return (((v ^ POLY) << 1) | 1) & 0xFFFFFFFF if v & ONE else (v << 1) & 0xFFFFFFFF


def unshift(v: int, nbytes: int) -> int:
    for _ in range(8 * nbytes):
        v = _xinv(v)
    return v


def region_batch(mem: bytes, bufs, inits):
    """Every buffer of a region batch through the model: chunk pass (raws and
    lane prefixes by lane_scan, Qe = the prefix at each event's lane), then
    the per-buffer fold."""
    NC = (len(mem) + 4095) // 4096
    mem = mem + bytes(NC * 4096 - len(mem))
    raws, pres = [], []
    for c in range(NC):
        raw, pre = lane_scan(piece_raws(mem[4096 * c:4096 * c + 4096]))
        raws.append(raw)
        pres.append(pre)
    qe = {}
    for s, L in bufs:
        for kind, c, o in region_events(s, s + L, L):
            qe[(kind, c, o)] = pres[c][o >> 6]
    return [region_fold_direct(mem, raws, qe, s, L, i) for (s, L), i in zip(bufs, inits)]


def chain_checkpoints(piece: bytes):
    """The chunk kernel's per-lane checkpoints: x_4c = S_4c ^ w[4c] (c = 1..3),
    S_k = raw(0, piece[0:4k)) -- the chain register before word 4c."""
    w = [int.from_bytes(piece[4 * k:4 * k + 4], "little") for k in range(16)]
    return [raw_bytes(0, piece[:16 * c]) ^ w[4 * c] for c in (1, 2, 3)]


def quad_prefix(x: int, quad: bytes, o: int) -> int:
    """crc32c_region_fold_kernel's quad_prefix: raw(0, piece[0:o)) from the
    checkpoint x (of word 4c, c = o >> 4) and the piece's 16-byte quad c."""
    c, m, r = o >> 4, (o >> 2) & 3, o & 3
    v = [int.from_bytes(quad[4 * j:4 * j + 4], "little") for j in range(4)]
    crc = (x ^ v[0]) if c else 0
    for j in range(m):
        crc = slice4(crc ^ v[j])
    cur = v[m]
    for b in range(r):
        crc = T[0][(crc ^ (cur >> (8 * b))) & 0xFF] ^ (crc >> 8)
    return crc


# ---- region path: the launch's partition (crc32c_dev_region.h run_region) ----
# Workgroup b of G owns the chunk range [B0, B1) = [nc b / G, nc (b+1) / G)
# and the buffers [I_b, I_b+1), I_b = the first buffer ending after chunk
# B0's start (I_0 = 0, I_G = n).  Its units: nfull two-chunk units, then
# single-chunk tail units, then the halo units re-streaming the chunks
# [C0, B0) of the one owned buffer that starts before B0.

def region_search(ends, A: int) -> int:
    """First buffer b with e_b > A (n when none), for non-decreasing ends."""
    for b, e in enumerate(ends):
        if e > A:
            return b
    return len(ends)


def region_units(nc: int, G: int, b: int, U: int = 2, rtail: int = 8):
    B0, B1 = nc * b // G, nc * (b + 1) // G
    cnt = B1 - B0
    nfull = (cnt - rtail) // U if cnt > rtail else 0
    return B0, B1, nfull, nfull + (cnt - nfull * U)


def region_span(u: int, B0: int, nfull: int, nunits: int, C0: int, nhalo: int, U: int = 2):
    """span_of(u): unit u's chunks (first, count) -- own units from [B0, B1),
    halo units from [C0, B0) once the halo is known."""
    if u < nunits:
        return (B0 + u * U, U) if u < nfull else (B0 + nfull * U + (u - nfull), 1)
    h = u - nunits
    if h >= nhalo:
        return B0, 0
    f = C0 + h * U
    return f, min(U, B0 - f)


def region_schedule(starts, lens, rel0: int, region_len: int, G: int, U: int = 2, rtail: int = 8, waves: int = 16):
    """Every workgroup's owned buffers and streamed chunks for a sorted,
    non-overlapping batch (starts relative to the region), asserting what the
    kernel relies on: every chunk a unit addresses lies in [0, nc) -- also in
    workgroups that own no chunk (G > nc) and for one-buffer batches; the
    owned ranges partition [0, n); every buffer's end lies in its owner's
    range and each of its chunks is streamed by its owner.  Returns, per
    workgroup, (owned buffer range, streamed chunk set)."""
    n = len(starts)
    nc = (rel0 + region_len + 4095) // 4096
    s = [rel0 + x for x in starts]
    ends = [x + L for x, L in zip(s, lens)]
    out, owned = [], []
    for b in range(G):
        B0, B1, nfull, nunits = region_units(nc, G, b, U, rtail)
        Ib = 0 if b == 0 else region_search(ends, B0 * 4096)
        Ib1 = n if b == G - 1 else region_search(ends, B1 * 4096)
        sb = s[Ib] if Ib < n else 0
        hc = B0 - (sb >> 12) if (Ib < Ib1 and sb < B0 * 4096) else 0
        nhalo, C0 = (hc + U - 1) // U, B0 - hc
        streamed = set()
        for u in range(nunits + nhalo + waves):  # + a count-0 unit per wave: the loop's exit pull
            f, c = region_span(u, B0, nfull, nunits, C0, nhalo, U)
            for k in range(c):
                assert 0 <= f + k < nc and C0 <= f + k < B1, (b, u, f, c, nc)
                streamed.add(f + k)
        assert streamed == set(range(C0, B1)), (b, C0, B1)
        for i in range(Ib, Ib1):
            if lens[i] >= REGION_DIRECT:
                assert B0 * 4096 < ends[i] <= B1 * 4096, (b, i)
                assert all(c in streamed for c in range(s[i] >> 12, (ends[i] - 1 >> 12) + 1)), (b, i)
        owned.extend(range(Ib, Ib1))
        out.append(((Ib, Ib1), streamed))
    assert owned == list(range(n))
    return out


def region_span_stale(u: int, B0: int, nfull: int, nunits: int, nhalo: int, hc: int, U: int = 2):
    """The round-4 form: first_of(u) with the halo origin C0 still at its
    initial B0 -- what a halo unit addressed when its first chunk was formed
    before its count had read the published halo."""
    if u < nunits:
        return region_span(u, B0, nfull, nunits, B0, 0, U)
    h = u - nunits
    return B0 + h * U, (min(U, hc - h * U) if h < nhalo else 0)


# ---- routed calls: the plan's verdict (crc32c_region.hip crc32c_route_plan,
# route_region) ------------------------------------------------------------
REGION_MAX_LEN = 128 << 10


def route_plan_bad(offs, lens, lim: int, base: int, pages: bool) -> bool:
    """The plan's bad flag over the whole batch (the OR of its partials):
    pairs out of order / overlapping, a length over REGION_MAX_LEN, a buffer
    outside [0, lim) and, with `pages` (batch_dev), a page of the span that
    holds no buffer byte -- the pairwise rule of the kernel, addresses
    A(x) = base + x."""
    M = (1 << 64) - 1
    n = len(offs)
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        e = (o + L) & M
        if e < o or L > REGION_MAX_LEN or o > lim or L > lim - o:
            return True
        if i + 1 < n:
            o1, L1 = int(offs[i + 1]), int(lens[i + 1])
            if e > o1:
                return True
            if pages:
                nz = L1 != 0
                pn = ((base + o1 - (0 if nz else 1)) & M) >> 12
                pe = ((base + e - 1) & M) >> 12
                if pn > pe + (1 if nz else 0):
                    return True
        if pages and i == 0 and L == 0:
            return True
    return False


def route_region_ok(offs, lens, lim: int, base: int, dyn: bool, cap_chunks: int) -> bool:
    """route_region: not bad, some bytes, and (dyn) the gap rule and the
    workspace's chunk cap over the span [offsets[0], end of the last)."""
    if route_plan_bad(offs, lens, lim, base, dyn):
        return False
    total = sum(min(int(x), REGION_MAX_LEN + 1) for x in lens)
    if total == 0:
        return False
    if not dyn:
        return True
    lo, hi = int(offs[0]), int(offs[-1]) + int(lens[-1])
    if hi - lo - total > total // 8 + 65536:
        return False
    O = (base + lo) & ~4095
    return (base + hi - O + 4095) // 4096 <= cap_chunks


def route_verdict(offs, lens, lim: int, base: int, dyn: bool, cap_chunks: int) -> str:
    """route_verdict: the region path for a region-shaped batch; else the
    page path when every buffer is exactly 4096 bytes ("pages_aligned" when
    every one is 16-byte aligned at A(x) = base + x); else the head + body
    kernels."""
    if route_region_ok(offs, lens, lim, base, dyn, cap_chunks):
        return "region"
    if all(int(x) == 4096 for x in lens):
        return "pages_aligned" if all((base + int(o)) % 16 == 0 for o in offs) else "pages"
    return "heads"


def span_pages_touched(offs, lens, base: int) -> bool:
    """Every 4 KiB page of the span [A(offsets[0]), A(end of the last)) holds
    a byte of some non-empty buffer (brute force)."""
    lo, hi = base + int(offs[0]), base + int(offs[-1]) + int(lens[-1])
    if hi <= lo:
        return True
    touched = set()
    for o, L in zip(offs, lens):
        if L:
            touched.update(range((base + int(o)) >> 12, ((base + int(o) + int(L) - 1) >> 12) + 1))
    return all(p in touched for p in range(lo >> 12, ((hi - 1) >> 12) + 1))


# ---- the compact LDS image (64 KiB; tools/diag/compact_steal.patch) ---------

def perm(s0: int, s1: int, sel: int) -> int:
    """v_perm_b32 for selector bytes 0..7 and 0x0C: bytes 0-3 of s1, 4-7 of
    s0, 0x0C gives 0x00."""
    src = s1.to_bytes(4, "little") + s0.to_bytes(4, "little")
    out = 0
    for i in range(4):
        c = (sel >> (8 * i)) & 0xFF
        out |= (src[c] if c < 8 else 0) << (8 * i)
    return out


def compact_image():
    """Dword image of kCLdsBytes as fill_compact_load/store write it: row b
    (256 B): slots j*8 + r = T[3 - j][b]; bytes 128.. of row 16n + v + 128h:
    T[n][v][32h + c] at dword 32 + c (lane 63's column left as the counter)."""
    img = [0] * 16384
    for b in range(256):
        for j in range(4):
            for r in range(8):
                img[b * 64 + j * 8 + r] = T[3 - j][b]
    for h in range(2):
        for n in range(8):
            for v in range(16):
                row = 16 * n + v + 128 * h
                for c in range(32):
                    img[row * 64 + 32 + c] = nibble_table(n, v, 32 * h + c)
    return img


def compact_lane_base(lane: int):
    r = (lane >> 2) & 7
    B = (r * 4) | ((8 + r) * 4) << 8 | ((16 + r) * 4) << 16 | ((24 + r) * 4) << 24
    sels = []
    for k in range(4):
        j = (k + lane) & 3
        sels.append(j | (4 + j) << 8 | 0x0C0C0000)
    return B, sels


def compact_slice4_addrs(x: int, lane: int):
    """Byte addresses of the four lookups of slice4c_next (k = 0..3)."""
    B, sels = compact_lane_base(lane)
    return [perm(x, B, s) for s in sels]


def compact_nibble_addrs(lr: int, lane: int):
    """Byte addresses of to_chunk_end_c's eight lookups (image + 128 + n*4096)."""
    jb = (lane & 31) << 2
    hb = 0x80808080 if lane >= 32 else 0
    lo = (lr & 0x0F0F0F0F) | hb
    hi = ((lr >> 4) & 0x0F0F0F0F) | hb
    out = []
    for n in range(8):
        src = lo if n % 2 == 0 else hi
        out.append(128 + n * 4096 + perm(src, jb, 0x0C0C0400 | (n // 2) << 8))
    return out
