"""Pure-Python model of the HIP engine's algorithm (test infrastructure).

Mirrors nvlevelz_amd/csrc/crc32c_kernels.hip step for step -- end-aligned
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


def chunk_raw(mem: bytes, p: int, L: int, J: int, c: int, s: int) -> int:
    """Raw register of chunk c of buffer [p, p+L) with ~init = s injected."""
    ce = p + L - CHUNK * (J - 1 - c)
    m = ce & 15
    lanes = []
    for lane in range(64):
        ps = ce - 64 * (64 - lane)
        a = ps - m
        # load_piece<false>: 16-byte vectors, skipped when wholly before p;
        # bytes of a loaded vector outside [p, e) are whatever memory holds.
        d = bytearray(80)
        for j in range(5):
            if (j < 4 or m != 0) and a + 16 * j + 16 > p:
                d[16 * j:16 * j + 16] = mem[a + 16 * j:a + 16 * j + 16]
        words = [int.from_bytes(d[m + 4 * k:m + 4 * k + 4], "little") for k in range(16)]
        if ce - CHUNK < p + 4:  # head: keep-mask bytes before p, inject ~init
            rel = max(-8, min(72, p - ps))
            for k in range(16):
                sh = rel - 4 * k
                keep = 0xFFFFFFFF if sh <= 0 else (0 if sh >= 4 else (0xFFFFFFFF << (8 * sh)) & 0xFFFFFFFF)
                inj = 0
                if 0 <= sh < 4:
                    inj = (s << (8 * sh)) & 0xFFFFFFFF
                elif -4 < sh < 0:
                    inj = s >> (-8 * sh)
                words[k] = (words[k] & keep) ^ inj
        crc = 0
        for w in words:
            crc = slice4(crc ^ w)
        lanes.append(crc)
    return wave_fold(lanes)


def batch(mem: bytes, bufs, inits, nwaves: int):
    """bufs: list of (p, L).  Returns final CRCs via waves + records + fix-up."""
    n = len(bufs)
    J = [1 if L <= CHUNK else (L + CHUNK - 1) // CHUNK for (_, L) in bufs]
    cs = [0]
    for j in J:
        cs.append(cs[-1] + j)
    Ttot = cs[-1]
    out = [None] * n
    recs = []
    NOBUF = -1
    for w in range(nwaves):
        t0, t1 = Ttot * w // nwaves, Ttot * (w + 1) // nwaves
        head, tail = (NOBUF, 0, 0, False), (NOBUF, 0, 0, False)
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
                            head = (i, acc, cnt, True)
                        cnt, from_zero = 0, True
                if c + 1 == J[i]:
                    i, c = i + 1, 0
                else:
                    c += 1
            if cnt:
                if from_zero:
                    tail = (i, acc, cnt, False)
                else:
                    head = (i, acc, cnt, False)
        recs.append((head, tail))
    # fix-up
    for w in range(nwaves):
        h = recs[w][0]
        if h[0] == NOBUF or not h[3]:
            continue
        total, after = h[1], h[2]
        for x in range(w - 1, -1, -1):
            hx, tx = recs[x]
            if hx[0] == h[0]:  # middle portion
                total ^= shift(hx[1], after * CHUNK)
                after += hx[2]
                continue
            if tx[0] == h[0]:  # first portion
                total ^= shift(tx[1], after * CHUNK)
                break
            assert hx[0] == NOBUF and tx[0] == NOBUF  # empty-range wave
        else:
            raise AssertionError("first portion not found")
        out[h[0]] = (~total) & 0xFFFFFFFF
    return out
