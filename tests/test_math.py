"""The GF(2) identities the HIP engine rests on, and a step-by-step model of
its decomposition (tests/kernel_model.py), checked against the oracle on the
CPU.  Catches a wrong butterfly order, end-alignment, masking, ~init
injection or wave-record fix-up before any GPU run."""
import random

import numpy as np
import pytest

import kernel_model as km


def test_slice_tables_match_oracle_steps(port):
    for b in range(256):
        assert km.T[0][b] == (km.raw_bytes(0, bytes([b])))
        for k in range(1, 4):
            assert km.T[k][b] == km.raw_bytes(0, bytes([b]) + bytes(k))


def test_shift_is_zero_feed():
    rng = random.Random(1)
    for _ in range(50):
        v = rng.getrandbits(32)
        n = rng.randrange(0, 300)
        assert km.shift(v, n) == km.raw_bytes(v, bytes(n))


def test_extend_identities(port):
    rng = random.Random(2)
    data = bytes(port.fill(77, 0, 20000))
    for _ in range(100):
        a = rng.randrange(0, 5000)
        b = rng.randrange(0, 5000)
        A, B = data[:a], data[a:a + b]
        init = rng.getrandbits(32)
        # Extend(init, D) = ~(shift(~init, |D|) ^ raw(0, D))
        want = port.extend(init, A)
        s = (~init) & 0xFFFFFFFF
        assert (~(km.shift(s, len(A)) ^ km.raw_bytes(0, A))) & 0xFFFFFFFF == want
        # raw(0, A||B) = shift(raw(0, A), |B|) ^ raw(0, B)
        assert km.raw_bytes(0, A + B) == km.shift(km.raw_bytes(0, A), len(B)) ^ km.raw_bytes(0, B)
        # crc(A||B) = shift(crc(A), |B|) ^ crc(B)   (standard combine)
        assert port.value(A + B) == km.shift(port.value(A), len(B)) ^ port.value(B)
        if len(A) >= 4:
            # state injection into the first word: raw(s, w||rest) = raw(0, (w^s)||rest)
            w = int.from_bytes(A[:4], "little") ^ s
            assert km.raw_bytes(s, A) == km.raw_bytes(0, w.to_bytes(4, "little") + A[4:])
        # leading zeros are invisible to a zero-state register
        assert km.raw_bytes(0, bytes(rng.randrange(0, 70)) + A) == km.raw_bytes(0, A)


def test_byte_sliced_operators():
    rng = random.Random(3)
    for op, dist in [(km.COMB[k], 64 << k) for k in range(6)] + [(km.SH4096, 4096)]:
        for _ in range(20):
            v = rng.getrandbits(32)
            assert km.apply_op(op, v) == km.shift(v, dist)


def test_fast_path_transposed_fold(port):
    """Fast path: load j puts bytes [1024j + 64b + 16a, +16) in lane (a, b) =
    (lane >> 4, lane & 15); the permlane32/permlane16 swap exchange across
    16-lane rows (row_transpose) leaves lane P holding piece P = bytes
    [64P, 64P+64); the butterfly over lane bits 0..5 uses distances 64*2^k."""
    data = bytes(port.fill(5, 0, 4096))
    # M[l][j] = (source lane, load) of the 16 B in lane l, slot j
    M = [[(l, j) for j in range(4)] for l in range(64)]

    def swap(M, ra, rb, half):
        """v_permlane{32,16}_swap on slot registers ra (vdst) and rb (src0):
        vdst's upper lanes of each 2*half group <-> src0's lower lanes."""
        out = [row[:] for row in M]
        for l in range(64):
            if (l // half) % 2 == 1:          # upper half of vdst swaps with lower half of src0
                out[l][ra] = M[l - half][rb]
                out[l - half][rb] = M[l][ra]
        return out
    M = swap(swap(M, 0, 2, 32), 1, 3, 32)
    M = swap(swap(M, 0, 1, 16), 2, 3, 16)
    lanes = []
    for l in range(64):
        src = [(sl >> 4, sl & 15, j) for (sl, j) in M[l]]  # (a, b, load) of each slot
        piece = b"".join(data[1024 * j + 64 * b + 16 * a:1024 * j + 64 * b + 16 * a + 16] for (a, b, j) in src)
        assert piece == data[64 * l:64 * l + 64]
        lanes.append(km.raw_bytes(0, piece))
    g = lanes
    for lev in range(6):
        pt = [g[l ^ (1 << lev)] for l in range(64)]
        g = [km.apply_op(km.COMB[lev], pt[l] if (l >> lev) & 1 else g[l]) ^ (g[l] if (l >> lev) & 1 else pt[l])
             for l in range(64)]
    assert len(set(g)) == 1 and g[0] == km.raw_bytes(0, data)
    assert (~km.raw_bytes(0xFFFFFFFF, data)) & 0xFFFFFFFF == port.value(data)


@pytest.mark.parametrize("seed", range(24))
def test_general_path_model(port, seed):
    """End-aligned chunks, masking, injection, per-wave ranges, records and
    fix-up, with more waves than chunks and buffers straddling waves."""
    rng = random.Random(seed)
    mem = bytes(port.fill(1000 + seed, 0, 120000))
    bufs, pos = [], 64
    for _ in range(rng.randrange(1, 7)):
        L = rng.choice([0, 1, 2, 3, 4, 5, 17, 63, 64, 65, 255, 256, 257, 1000, 1024, 1025, 3000, 4095, 4096, 4097,
                        4100, 4109, 4112, 4113, 4156, 4196, 4396, 6096, 8191, 8192, 8208, 8209, 9000, 13000, 20000])
        pos += rng.randrange(0, 40)
        bufs.append((pos, L))
        pos += L
    inits = [rng.getrandbits(32) for _ in bufs]
    nw = rng.choice([1, 2, 3, 5, 16, 33])
    got = km.batch(mem, bufs, inits, nw)
    want = [port.extend(i, mem[a:a + L]) for (a, L), i in zip(bufs, inits)]
    assert got == want


def test_alignment_sweep_model(port):
    """Every start alignment mod 16 x lengths around the chunk boundaries
    through the model, with garbage before and after each buffer; the model
    also asserts that no load touches a 16-byte granule without buffer bytes
    (fault safety) -- or, for a long head's straddling row slot, bytes outside
    its granule's page."""
    mem = bytes(port.fill(0xA11, 0, 200000))
    lens = [4, 5, 6, 7, 15, 16, 17, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 4095, 4096, 4097, 4098, 4099,
            4100, 4101, 4108, 4111, 4112, 4113, 4114, 4160, 4161, 4352, 4353, 5120, 5121, 8191, 8207, 8208, 8209,
            8210, 8212]
    for a in range(16):
        bufs = []
        pos = 4096 + a
        for L in lens:
            bufs.append((pos, L))
            pos += L + 16 * 7 + 3
        inits = [(0x1F2E3D4C * (k + 1) + a) & 0xFFFFFFFF for k in range(len(bufs))]
        got = km.batch(mem, bufs, inits, 1)
        want = [port.extend(i, mem[p:p + L]) for (p, L), i in zip(bufs, inits)]
        assert got == want, a


@pytest.mark.parametrize("page_off", [0, 4, 15, 16, 17, 28, 4079, 4080])
def test_long_head_model(port, page_off):
    """Long heads (1025..4095 bytes, run_heads -> long_heads) at starts around a
    4 KiB page boundary: buffers starting in a page's first granule take the
    lane-group path (head_raw), the rest the whole-chunk path (long_head_raw,
    whose straddling row slot must stay in its granule's page)."""
    mem = bytes(port.fill(0x10E6, 0, 64 * 4096))
    rng = random.Random(page_off)
    for k in range(40):
        hl = rng.choice([1025, 1026, 1027, 1028, 1100, 2047, 2048, 2049, 3000, 4000, 4080, 4081, 4092, 4094, 4095])
        J = rng.choice([1, 1, 2, 3])
        L = hl + 4096 * (J - 1)
        p = 4096 * (2 + 13 * k % 40) + page_off
        s = rng.getrandbits(32)
        assert km.long_head(p, hl) == (((p >> 4) & 255) != 0)
        got = km.chunk_raw(mem, p, L, J, 0, s)
        assert got == km.raw_bytes(0, bytes(4096 - hl) + bytes(b ^ ((s >> (8 * q)) & 0xFF) if q < 4 else b
                                                              for q, b in enumerate(mem[p:p + hl]))), (p, hl)


@pytest.mark.parametrize("page_off", [0, 1, 4, 13, 15, 16, 17, 28, 4079, 4080])
def test_masked_pass_model(port, page_off):
    """kMasked scheduler-A passes (fixed batches of one 1025..4095-byte chunk
    per buffer) at starts around a 4 KiB page boundary, page-first granules
    included (page_head_words): loads stay in the buffer's granules or in its
    first granule's page, and the register matches the reference."""
    mem = bytes(port.fill(0x3A5C, 0, 64 * 4096))
    rng = random.Random(1000 + page_off)
    for k in range(30):
        L = rng.choice([1025, 1026, 1027, 1028, 1100, 2047, 2048, 2049, 3000, 3500, 4000, 4080, 4092, 4095])
        p = 4096 * (2 + 13 * k % 40) + page_off
        s = rng.getrandbits(32)
        got = km.masked_pass_raw(mem, p, L, s)
        want = km.raw_bytes(0, bytes(4096 - L) + bytes(b ^ ((s >> (8 * q)) & 0xFF) if q < 4 else b
                                                       for q, b in enumerate(mem[p:p + L])))
        assert got == want, (p, L)


def test_unshift_inverts_shift():
    rng = random.Random(9)
    for _ in range(40):
        v = rng.getrandbits(32)
        n = rng.randrange(0, 300)
        assert km.unshift(km.shift(v, n), n) == v


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_region_path_model(port, seed):
    """The region decomposition (page-aligned chunks, Qe at event lanes,
    piece-prefix re-reads, per-buffer fold with ~init at the start) against
    the oracle: packed, gapped, chunk- and piece-boundary starts/ends, tiny
    buffers and multi-chunk buffers."""
    rng = random.Random(100 + seed)
    mem = bytes(port.fill(seed + 5, 0, 3 * 4096 * 4 + 512))
    bufs, inits = [], []
    p = rng.randrange(0, 200)
    specials = [4096 - 3, 4096, 64, 63, 0, 1, 2, 3, 4097, 8192 + 5, 128]
    while True:
        L = specials.pop() if specials else rng.choice([rng.randrange(0, 70), rng.randrange(64, 5000),
                                                       rng.randrange(4000, 9000)])
        if p + L > len(mem):
            break
        bufs.append((p, L))
        inits.append(rng.getrandbits(32) if rng.random() < 0.5 else 0)
        p += L + rng.choice([0, 0, 4, 5, 1, 64 - (p + L) % 64])
    # starts/ends exactly on piece and chunk boundaries; two whole chunks
    # (L = 8192: the longest buffer the direct fold takes); three chunks
    # and the long fold's steps of up to four chunks: 3..12 chunks, chunk-aligned ends too
    bufs += [(4096, 64), (4096 * 2 - 64, 64 + 4096), (4096, 8192), (100, 8192), (4095, 4098),
             (17, 4096 * 5), (4096, 4096 * 5), (300, 4096 * 9 + 77), (5, 4096 * 12 - 5), (4100, 4096 * 4 + 8)]
    inits += [0, 7, 3, 0, 9, 1, 2, 0, 5, 6]
    got = km.region_batch(mem, bufs, inits)
    want = [port.extend(i, mem[s:s + L]) for (s, L), i in zip(bufs, inits)]
    assert got == want


def test_region_lane_scan(port):
    """The region kernel's chunk step: per-lane nibble-table shifts to the
    chunk end + XOR scan give the chunk raw and, at every lane L, the masked
    butterfly Qe(L) (the chunk bytes [0, 64L) at the chunk end)."""
    rng = random.Random(21)
    for _ in range(3):
        chunk = bytes(rng.getrandbits(8) for _ in range(4096))
        lr = km.piece_raws(chunk)
        raw, pre = km.lane_scan(lr)
        assert raw == km.raw_bytes(0, chunk) == km.wave_fold(lr)
        for L in range(64):
            assert pre[L] == km.masked_fold(lr, L), L


def test_region_quad_prefix_from_checkpoints(port):
    """The fold kernel's R(p) from the chunk kernel's chain checkpoint and one
    16-byte quad equals the piece prefix's raw at every offset 0..63."""
    rng = random.Random(12)
    for _ in range(20):
        piece = bytes(rng.getrandbits(8) for _ in range(64))
        cps = km.chain_checkpoints(piece)
        for o in range(64):
            c = o >> 4
            x = cps[c - 1] if c else 0
            assert km.quad_prefix(x, piece[16 * c:16 * c + 16], o) == km.raw_bytes(0, piece[:o]), o


def _grid_for(nc: int, num_cu: int = 256) -> int:
    return max(1, min(num_cu, -(-nc // 16)))  # crc32c_launch.h grid_for


@pytest.mark.parametrize("G", [None, 1, 4, 16, 256])
@pytest.mark.parametrize("case", ["one_block", "one_block_lead", "one_mib", "one_tiny", "r_shape", "cfg3_like"])
def test_region_schedule_bounds(case, G):
    """run_region's partition over the grid (tests/kernel_model.py
    region_schedule): every chunk address of every unit -- own, tail, halo
    and the count-0 units the waves pull on their way out -- lies inside the
    region's chunks, including one-buffer batches (test_gpu_region's n = 1
    cases) and grids with more workgroups than chunks (workgroups that own
    no chunk); the owned buffer ranges partition the batch and each buffer's
    chunks are streamed by its owner.  G None: the launcher's own grid."""
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    if case == "one_block":
        starts, lens, rel0 = [0], [4097], 0
    elif case == "one_block_lead":
        starts, lens, rel0 = [int(rng.integers(0, 16))], [int(rng.integers(3364, 4110))], 7
    elif case == "one_mib":
        starts, lens, rel0 = [5], [1 << 20], 100
    elif case == "one_tiny":
        starts, lens, rel0 = [3], [9], 4090
    elif case == "r_shape":
        lens = rng.integers(3364, 4110, 3000).tolist()
        starts = (np.cumsum([0] + [L + 4 for L in lens[:-1]])).tolist()
        rel0 = 11
    else:
        lens = (512 + rng.integers(0, 65025, 400)).tolist()
        starts = (np.cumsum([0] + lens[:-1])).tolist()
        rel0 = 0
    region_len = starts[-1] + lens[-1] + 3
    nc = (rel0 + region_len + 4095) // 4096
    km.region_schedule(starts, lens, rel0, region_len, G or _grid_for(nc))


def test_region_stale_halo_origin_addresses_past_the_region():
    """The fault of a round-4 variant: a halo unit whose first
    chunk was formed from the halo origin's initial value B0 (before the
    published halo was read) addresses chunks past the region when the halo
    is longer than the workgroup's own range -- one buffer spanning many
    workgroups' ranges, owned by the last one.  span_of (the shipped form)
    reads the halo first (test_region_schedule_bounds)."""
    starts, lens, rel0 = [5], [1 << 20], 100
    nc = (rel0 + starts[0] + lens[0] + 4095) // 4096
    G = 16
    B0, B1, nfull, nunits = km.region_units(nc, G, G - 1)
    hc = B0 - ((rel0 + starts[0]) >> 12)
    nhalo = (hc + 1) // 2
    addr = [f + k for u in range(nunits, nunits + nhalo)
            for f, c in [km.region_span_stale(u, B0, nfull, nunits, nhalo, hc)] for k in range(c)]
    assert max(addr) >= nc  # past the region: the illegal address
    km.region_schedule(starts, lens, rel0, lens[0] + starts[0], G)  # the shipped span_of stays inside


def test_compact_image_lookups_and_banks():
    """The 64 KiB image of tools/diag/compact_steal.patch (two workgroups per
    CU; measured, not shipped -- DESIGN §8): each lane's four slice
    lookups (bytes taken in the lane's rotated order) sum to slice4(x), its
    eight nibble lookups to the lane's shift to the chunk end, and every
    ds_read_b32 of a wave hits 32 distinct banks ((a/4) mod 32) in each
    32-lane group, whatever the data."""
    img = km.compact_image()
    rng = random.Random(5)
    for trial in range(40):
        xs = [rng.getrandbits(32) for _ in range(64)]
        addrs = [km.compact_slice4_addrs(xs[l], l) for l in range(64)]
        for l in range(64):
            a = addrs[l]
            assert all(0 <= v < 65536 and v % 4 == 0 and (v & 255) < 128 for v in a)
            got = 0
            for v in a:
                got ^= img[v // 4]
            assert got == km.slice4(xs[l])
        for k in range(4):
            for g in (range(32), range(32, 64)):
                assert len({(addrs[l][k] // 4) % 32 for l in g}) == 32
        nad = [km.compact_nibble_addrs(xs[l], l) for l in range(64)]
        for l in range(63):  # lane 63: identity, its column is the counter
            got = 0
            for v in nad[l]:
                assert 0 <= v < 65536 and (v & 255) >= 128
                got ^= img[v // 4]
            assert got == km.shift(xs[l], 64 * (63 - l))
        for n in range(8):
            for g in (range(32), range(32, 64)):
                assert len({(nad[l][n] // 4) % 32 for l in g}) == 32
    ctr = (128 * 256 + 128 + 31 * 4) // 4  # kCCtrOff: lane 63's slot, row (n=0, v=0, h=1)
    assert ctr == 128 * 64 + 32 + 31


def test_region_long_fold_runs():
    """The cooperative fold of a long region buffer (tools/diag/long_fold.patch,
    measured and not shipped -- DESIGN §8 item 0): items
    0..nit-1 (the head term, then the middle chunks' raws) split into 8
    runs [ceil(nit q / 8), ceil(nit (q+1) / 8)) -- run 0 always holds item 0
    --, each run's Horner times x^(8*4096*(nit - end + 1)), XORed, equals the
    per-lane chain acc = shift4096(acc) ^ item, shifted once more (fold_out's
    longer branch)."""
    rng = random.Random(11)
    for nit in list(range(2, 34)) + [40, 63]:
        items = [rng.getrandbits(32) for _ in range(nit)]
        acc = items[0]
        for t in range(1, nit):
            acc = km.shift(acc, 4096) ^ items[t]
        acc = km.shift(acc, 4096)
        got = 0
        for q in range(8):
            a, b = (nit * q + 7) // 8, (nit * (q + 1) + 7) // 8
            if q == 0:
                assert a == 0 and b >= 1
            if b <= a:
                continue
            P = items[a]
            for t in range(a + 1, b):
                P = km.shift(P, 4096) ^ items[t]
            got ^= km.shift(P, 4096 * (nit - b + 1))
        assert got == acc, nit
