"""CPU checks of the fp32 Winograd F(4x4, 3x3) conv path (csrc/kernels/conv_wino4_f32.hip): the host
weight transform + fragment packing (ops/conv.py wino4_pack_np) unpacked with the kernel's exact lane /
element indexing, the split input / output transforms of the two waves of a pair (B^T rows 0-2 / 3-5,
A^T columns 0-2 / 3-5) transcribed formula by formula, and the wave-image bookkeeping (segments, 9-unit
column groups, the DMA source table, every lane's patch reads) -- all against a direct 3x3 / stride-1 /
pad-1 convolution, on the ResNet stage shapes and odd maps.  Parity with the reference's Keras float32
3x3 convs: `/root/reference/test/test.py:13`."""
import numpy as np
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C

from test_wino import direct_conv


def _bt(d0, d1, d2, d3, d4, d5):
    """conv_wino4_f32.hip w4_bt."""
    s12, s34, m12, m43, m13, m42 = d1 + d2, d3 + d4, d1 - d2, d4 - d3, d1 - d3, d4 - d2
    return (4 * d0 - 5 * d2 + d4, -4 * s12 + s34, 4 * m12 + m43, -2 * m13 + m42, 2 * m13 + m42,
            4 * d1 - 5 * d3 + d5)


def _colh(h, e):
    """w4_colh<H>: B^T rows 3h .. 3h + 2 on the 5 row-transformed patch rows h .. h + 4."""
    e0, e1, e2, e3, e4 = e
    if h == 0:
        return (4 * e0 - 5 * e2 + e4, -4 * (e1 + e2) + (e3 + e4), 4 * (e1 - e2) + (e4 - e3))
    m13, m42 = e0 - e2, e3 - e1
    return (-2 * m13 + m42, 2 * m13 + m42, 4 * e0 - 5 * e2 + e4)


def _at(m):
    """w4_at."""
    s12, d12, s34, d34 = m[1] + m[2], m[1] - m[2], m[3] + m[4], m[3] - m[4]
    return (m[0] + s12 + s34, 2 * d34 + d12, 4 * s34 + s12, 8 * d34 + d12 + m[5])


def _epi_w(h, m0, m1, m2):
    """The epilogue's partial A^T column stage of wave h (rows pa = 3h .. 3h + 2 of M)."""
    if h == 0:
        s12, d12 = m1 + m2, m1 - m2
        return (m0 + s12, d12, s12, d12)
    s34, d34 = m0 + m1, m0 - m1
    return (s34, 2 * d34, 4 * s34, 8 * d34 + m2)


def test_split_transforms_are_the_full_transforms():
    rng = np.random.default_rng(0)
    d = rng.standard_normal((6, 6))
    full = C.WINO4_BT @ d @ C.WINO4_BT.T
    rows = np.array([_bt(*d[i]) for i in range(6)])                       # row transforms (over dx)
    for h in (0, 1):
        for pb in range(6):
            got = _colh(h, rows[h:h + 5, pb])
            assert np.allclose(got, full[3 * h:3 * h + 3, pb])
    m = rng.standard_normal((6, 6))
    want = C.WINO4_AT @ m @ C.WINO4_AT.T
    got = np.zeros((4, 4))
    for h in (0, 1):
        w = np.array([_epi_w(h, *m[3 * h:3 * h + 3, pb]) for pb in range(6)]).T    # [a][pb]
        got += np.array([_at(w[a]) for a in range(4)])
    assert np.allclose(got, want)
    assert np.allclose(np.array([_at(m[:, j]) for j in range(6)]).T, C.WINO4_AT @ m)


def _unpack(packed):
    """U[p][c][n] from the packed tensor, read as the kernel does: lane l = 16 q + n' of position p of
    chunk kc of channel group cg, element (j, s) -> c = 8 kc + 2 q + s, n = 32 cg + 16 j + n'."""
    NG, KC = packed.shape[:2]
    U = np.zeros((36, KC * 8, NG * 32))
    for cg in range(NG):
        for kc in range(KC):
            for lane in range(64):
                q, n_ = lane >> 4, lane & 15
                for j in range(2):
                    for s in range(2):
                        U[:, 8 * kc + 2 * q + s, 32 * cg + 16 * j + n_] = packed[cg, kc, :, lane, j, s]
    return U


@pytest.mark.parametrize("H,W,Ci,N", [(8, 8, 16, 32), (7, 7, 32, 32), (6, 10, 16, 64), (14, 14, 16, 32)])
def test_wino4_packing_and_split_arithmetic_match_direct_conv(H, W, Ci, N):
    rng = np.random.default_rng(H * 100 + Ci)
    B = 2
    x = rng.standard_normal((B, H, W, Ci))
    k = rng.standard_normal((3, 3, Ci, N)) / np.sqrt(9 * Ci)
    packed = C.wino4_pack_np(k)
    assert packed.shape == (N // 32, Ci // 8, 36, 64, 2, 2) and packed.dtype == np.float32
    U = _unpack(packed.astype(np.float64))
    TH, TW = (H + 3) // 4, (W + 3) // 4
    xp = np.zeros((B, 4 * TH + 2, 4 * TW + 2, Ci))
    xp[:, 1:H + 1, 1:W + 1] = x
    y = np.zeros((B, 4 * TH, 4 * TW, N))
    for ty in range(TH):
        for tx in range(TW):
            d = xp[:, 4 * ty:4 * ty + 6, 4 * tx:4 * tx + 6]                 # [B][6][6][C]
            out = np.zeros((B, 4, 4, N))
            for h in (0, 1):
                rows = np.stack([np.stack(_bt(*[d[:, h + rr, dx] for dx in range(6)]), 1)
                                 for rr in range(5)], 1)                     # [B][5 rows][6 pb][C]
                V = np.stack([np.stack(_colh(h, [rows[:, rr, pb] for rr in range(5)]), 1)
                              for pb in range(6)], 2)                        # [B][3 pa][6 pb][C]
                M = np.einsum("bapc,apcn->bapn", V, U.reshape(6, 6, Ci, N)[3 * h:3 * h + 3])
                w = np.stack([np.stack(_epi_w(h, M[:, 0, pb], M[:, 1, pb], M[:, 2, pb]), 1)
                              for pb in range(6)], 2)                        # [B][4 a][6 pb][N]
                for a in range(4):
                    out[:, a] += np.stack(_at([w[:, a, pb] for pb in range(6)]), 1)
            y[:, 4 * ty:4 * ty + 4, 4 * tx:4 * tx + 4] = out
    got = y[:, :H, :W]
    want = direct_conv(x, k)
    assert np.abs(got - want).max() / np.abs(want).max() < 5e-6


def test_wino4_pack_rejects_other_filters():
    with pytest.raises(ValueError):
        C.wino4_pack_np(np.zeros((1, 1, 16, 32), np.float32))
    with pytest.raises(ValueError):
        C.wino4_pack_np(np.zeros((3, 3, 8, 32), np.float32))
    with pytest.raises(ValueError):
        C.wino4_pack_np(np.zeros((3, 3, 16, 48), np.float32))


def test_pack_conv_f32_attaches_wino4():
    k3 = np.random.default_rng(0).standard_normal((3, 3, 32, 64)).astype(np.float32)
    pc = C.pack_conv_f32(k3, np.zeros(64, np.float32), 1, ((1, 1), (1, 1)), "cpu")
    assert pc.wino4 is not None and tuple(pc.wino4.shape) == (2, 4, 36, 64, 2, 2)
    assert C.f32_cfg_supported(200, 32, 64, pc)
    k48 = np.zeros((3, 3, 32, 48), np.float32)
    assert C.pack_conv_f32(k48, np.zeros(48, np.float32), 1, ((1, 1), (1, 1)), "cpu").wino4 is None
    assert C.wino4_splits(64) == [1, 2, 4] and C.wino4_splits(512) == [1, 2, 4, 8] and C.wino4_splits(16) == [1]


# --- the wave image -------------------------------------------------------------------------------

def _segments(tw0, T, TW, align):
    """conv_wino4_f32.hip: (lo, pitch) per tile-row segment of tiles tw0 .. tw0 + 15 and the bases
    (align: each next segment starts on the 16-B bank slot 9 x (tiles before it) mod 16)."""
    tlast = min(tw0 + 15, T - 1)
    R0 = tw0 // TW
    nseg = tlast // TW - R0 + 1 if tw0 < T else 0
    lo_, pitch, base = [], [], [0]
    r0 = 0
    for sg in range(8):
        lo = tw0 - R0 * TW if sg == 0 else 0
        hi = tlast - (R0 + sg) * TW if sg == nseg - 1 else TW - 1
        n = hi - lo + 1 if sg < nseg else 0
        lo_.append(lo)
        pitch.append(9 * n + 4 if n else 0)
        r0 += n
        b = base[-1] + 6 * pitch[-1]
        base.append(b + ((9 * r0 - b) & 15) if align and sg + 1 < nseg else b)
    return R0, nseg, lo_, pitch, base


def _plan(B, H, W):
    """conv_wino4_pieces: (pieces, align), aligned bases preferred while they fit in 19 pieces."""
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    for align in (1, 0):
        need = max(_segments(tw0, T, TW, align)[4][8] for tw0 in range(0, T, 16))
        pieces = max(15, -(-need // 64))
        if pieces <= 19:
            return pieces, align
    return 0, 0


def _image_maps(tw0, B, H, W, pieces, align):
    """The kernel's DMA source table (unit -> (img, iy, ix, half) or None) and every lane's patch reads
    ((r, q, dy, dx) -> (unit, 8-byte half)) for the tile group starting at tile tw0."""
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    R0, nseg, lo_, pitch, base = _segments(tw0, T, TW, align)
    units = base[8]
    hp = (pieces + 1) // 2
    dma = {}
    for h in (0, 1):
        for ii in range(hp):
            i = 2 * ii + h
            if i >= pieces:
                continue                                # the odd last piece belongs to wave 0
            for lane in range(64):
                u = i * 64 + lane
                sg = sum(1 for k in range(1, 8) if u >= base[k])
                local = u - base[sg]
                row = local // pitch[sg] if pitch[sg] else 0
                uu = local - row * pitch[sg]
                g9, e = divmod(uu, 9)
                px, hh = 4 * g9 + (e >> 1), e & 1
                R = R0 + sg
                im, ty = divmod(R, TH)
                iy, ix = 4 * ty - 1 + row, 4 * lo_[sg] - 1 + px
                ok = u < units and e != 8 and R < B * TH and 0 <= iy < H and 0 <= ix < W
                assert u not in dma
                dma[u] = (im, iy, ix, hh) if ok else None
    reads = {}
    for r in range(16):
        t = tw0 + r
        if t >= T:
            continue
        tsg = t // TW - R0
        cgl = t - (R0 + tsg) * TW - lo_[tsg]
        prs = pitch[tsg] * 16
        for q in range(4):
            for h in (0, 1):
                prd = (base[tsg] + 9 * cgl + (q >> 1)) * 16 + 8 * (q & 1) + h * prs
                for row in range(5):
                    for dx in range(6):
                        off = prd + row * prs + 16 * (2 * dx if dx < 4 else 2 * dx + 1)
                        reads[(r, q, h + row, dx, h)] = (off // 16, (off % 16) // 8)
    return dma, reads, units


SHAPES = [(32, 56, 56), (32, 28, 28), (32, 14, 14), (32, 7, 7), (3, 9, 13), (2, 8, 8), (5, 12, 7)]


@pytest.mark.parametrize("B,H,W", SHAPES)
def test_wino4_wave_image_bookkeeping(B, H, W):
    """Every lane's patch pixels come from the image units that the pair's LDS-DMA filled with exactly
    that input pixel and channel half (zeros outside the map), within the staged pieces, for every tile
    group; the host's plan (pieces, bank-aligned bases) is the one transcribed here."""
    pieces, align = _plan(B, H, W)
    assert 15 <= pieces <= 19
    assert tuple(C.kernels().conv_wino4_pieces(B, H, W)) == (pieces, align)
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    for tw0 in range(0, T, 16):
        dma, reads, units = _image_maps(tw0, B, H, W, pieces, align)
        assert units <= pieces * 64
        for (r, q, dy, dx, h), (u, half8) in reads.items():
            t = tw0 + r
            im, rem = divmod(t, TH * TW)
            ty, tx = divmod(rem, TW)
            iy, ix = 4 * ty - 1 + dy, 4 * tx - 1 + dx
            want = (im, iy, ix, q >> 1) if 0 <= iy < H and 0 <= ix < W else None
            assert half8 == (q & 1)
            assert dma[u] == want, (tw0, r, q, dy, dx)


@pytest.mark.parametrize("B,H,W,worst_ok", [(32, 56, 56, 2), (32, 28, 28, 3), (32, 14, 14, 1), (32, 7, 7, 1)])
def test_wino4_patch_read_bank_conflicts(B, H, W, worst_ok):
    """ds_read_b64 serves lanes 0-31 and 32-63 in one LDS cycle each when their 8-byte words fall on
    distinct banks (MI355X_MICROARCH.md LDS table).  With 9-unit column groups the tiles of one segment
    take distinct 16-B slots; the aligned segment bases make full-row tile groups (stages 4 / 5 at
    bs 32) conflict-free; partial segments of a different pitch (stages 2 / 3) still meet a few."""
    pieces, align = _plan(B, H, W)
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    worst = 0
    for tw0 in range(0, T, 16):
        _, reads, _ = _image_maps(tw0, B, H, W, pieces, align)
        for h in (0, 1):
            for dy in range(h, h + 5):
                for dx in range(6):
                    for half in (0, 1):                 # lane groups {q = 0, 1} and {q = 2, 3}
                        banks = {}
                        for r in range(16):
                            for q in (2 * half, 2 * half + 1):
                                key = (r, q, dy, dx, h)
                                if key not in reads:
                                    continue
                                u, h8 = reads[key]
                                for w in range(2):
                                    bank = ((u * 16 + 8 * h8) // 4 + w) % 64
                                    banks.setdefault(bank, set()).add((u, h8))
                        worst = max(worst, max(len(v) for v in banks.values()))
    assert worst <= worst_ok
