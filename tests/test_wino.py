"""CPU checks of the fp32 Winograd F(2x2, 3x3) conv path (csrc/kernels/conv_wino_f32.hip):
the host weight transform + fragment packing (ops/conv.py wino_pack_np), unpacked with the exact
lane / element indexing the kernel uses, and the input / output transforms, reproduce a direct
3x3 / stride-1 / pad-1 convolution (even and odd maps: ResNet stages 2-4 and stage 5's 7x7)."""
import numpy as np
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C


def direct_conv(x, k):
    B, H, W, Ci = x.shape
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1), (0, 0)))
    y = np.zeros((B, H, W, k.shape[3]))
    for i in range(3):
        for j in range(3):
            y += np.einsum("bhwc,cn->bhwn", xp[:, i:i + H, j:j + W], k[i, j])
    return y


def kernel_emulation(x, packed):
    """The kernel's arithmetic in fp64: U_p[c][n] read as lane l = 16 q + n', element s of piece
    (kc, nf, p); V = B^T d B per 4x4 patch; y = A^T (sum_c V U) A, cropped to the map."""
    B, H, W, Ci = x.shape
    KC, NF = packed.shape[0], packed.shape[1]
    N = NF * 16
    U = np.zeros((16, Ci, N))
    for kc in range(KC):
        for nf in range(NF):
            for p in range(16):
                for lane in range(64):
                    q, n_ = lane >> 4, lane & 15
                    for s in range(4):
                        U[p, 16 * kc + 4 * q + s, 16 * nf + n_] = packed[kc, nf, p, lane, s]
    TH, TW = (H + 1) // 2, (W + 1) // 2
    xp = np.zeros((B, 2 * TH + 2, 2 * TW + 2, Ci))
    xp[:, 1:H + 1, 1:W + 1] = x
    y = np.zeros((B, 2 * TH, 2 * TW, N))
    BT, AT = C.WINO_BT, C.WINO_AT
    for ty in range(TH):
        for tx in range(TW):
            d = xp[:, 2 * ty:2 * ty + 4, 2 * tx:2 * tx + 4]                  # [B][4][4][C]
            V = np.einsum("ai,bijc,dj->badc", BT, d, BT).reshape(B, 16, Ci)  # p = 4a + b
            M = np.einsum("bpc,pcn->bpn", V, U).reshape(B, 4, 4, N)
            y[:, 2 * ty:2 * ty + 2, 2 * tx:2 * tx + 2] = np.einsum("ai,bijn,dj->badn", AT, M, AT)
    return y[:, :H, :W]


@pytest.mark.parametrize("H,W,Ci,N", [(8, 8, 32, 16), (7, 7, 16, 32), (6, 10, 16, 16)])
def test_wino_packing_and_transforms_match_direct_conv(H, W, Ci, N):
    rng = np.random.default_rng(H * 100 + Ci)
    x = rng.standard_normal((2, H, W, Ci))
    k = rng.standard_normal((3, 3, Ci, N)) / np.sqrt(9 * Ci)
    packed = C.wino_pack_np(k)
    assert packed.shape == (Ci // 16, N // 16, 16, 64, 4) and packed.dtype == np.float32
    got = kernel_emulation(x, packed.astype(np.float64))
    want = direct_conv(x, k)
    # the packed weights are fp32: agreement to fp32 rounding of U
    assert np.abs(got - want).max() / np.abs(want).max() < 2e-6


def test_wino_pack_rejects_other_filters():
    with pytest.raises(ValueError):
        C.wino_pack_np(np.zeros((1, 1, 16, 16), np.float32))
    with pytest.raises(ValueError):
        C.wino_pack_np(np.zeros((3, 3, 8, 16), np.float32))


def test_pack_conv_f32_attaches_wino_only_to_3x3_s1_p1():
    k3 = np.random.default_rng(0).standard_normal((3, 3, 32, 64)).astype(np.float32)
    pc = C.pack_conv_f32(k3, np.zeros(64, np.float32), 1, ((1, 1), (1, 1)), "cpu")
    assert pc.wino is not None and tuple(pc.wino.shape) == (2, 4, 16, 64, 4)
    assert C.f32_cfg_supported(80, 32, 64, pc) and not C.f32_cfg_supported(84, 32, 64, pc)   # 64 % 48
    pc2 = C.pack_conv_f32(k3, np.zeros(64, np.float32), 2, ((0, 1), (0, 1)), "cpu")
    assert pc2.wino is None and not C.f32_cfg_supported(80, 32, 64, pc2)
    k1 = np.zeros((1, 1, 32, 64), np.float32)
    assert C.pack_conv_f32(k1, np.zeros(64, np.float32), 1, ((0, 0), (0, 0)), "cpu").wino is None


def _wino_sw(slot):
    """conv_wino_f32.hip wino_sw: the bank swizzle of the v2 wave image (cfgs 103-105)."""
    row = slot >> 4
    return slot ^ ((2 * row + 8 * (row >> 2)) & 15)


def _v2_lane_maps(tw0, T, TW, TH, H, W, sw=False):
    """conv_wino_f32_v2_kernel's wave-image bookkeeping, transcribed: the LDS-DMA source of every
    (piece, lane) slot and every lane's patch pixel index; returns (dma, reads) for checking.
    With `sw` the DMA of LDS slot S fetches logical slot wino_sw(S), and dma is keyed by LDS slot."""
    TR_ = T // TW
    tlast = min(tw0 + 15, T - 1)
    R0 = tw0 // TW
    nseg = tlast // TW - R0 + 1 if tw0 < T else 0
    seg_lo, seg_w, seg_b = [], [], [0]
    for sg in range(4):
        lo = tw0 - R0 * TW if sg == 0 else 0
        hi = tlast - (R0 + sg) * TW if sg == nseg - 1 else TW - 1
        seg_lo.append(lo)
        seg_w.append(2 * (hi - lo + 1) + 2 if sg < nseg else 0)
        seg_b.append(seg_b[-1] + 4 * seg_w[-1])
    dma = {}
    for i in range(10):
        for lane in range(64):
            sl = _wino_sw(i * 64 + lane) if sw else i * 64 + lane
            pix, qq = sl >> 2, sl & 3
            sg = sum(1 for k in (1, 2, 3) if pix >= seg_b[k])
            wdt, lo, bb = seg_w[sg], (seg_lo[0] if sg == 0 else 0), seg_b[sg]
            lp = pix - bb
            prow = lp // wdt if wdt else 0
            pcol = lp - prow * wdt
            R = R0 + sg
            img, ty = R // TH, R % TH
            iy, ix = 2 * ty - 1 + prow, 2 * lo - 1 + pcol
            inside = pix < seg_b[4] and R < TR_ and 0 <= iy < H and 0 <= ix < W
            dma[i * 64 + lane] = (img, iy, ix) if inside else None
    reads = {}
    for r in range(16):
        t = tw0 + r
        if t >= T:
            continue
        tsg = t // TW - R0
        prow0 = seg_b[tsg] + 2 * (t - (R0 + tsg) * TW - (seg_lo[0] if tsg == 0 else 0))
        for dy in range(4):
            for dx in range(4):
                reads[(r, dy, dx)] = prow0 + dy * seg_w[tsg] + dx
    return dma, reads, seg_b[4]


@pytest.mark.parametrize("sw", [False, True])
@pytest.mark.parametrize("B,H,W", [(3, 56, 56), (2, 28, 28), (3, 14, 14), (5, 7, 7), (2, 9, 13), (2, 8, 8)])
def test_wino_v2_wave_image_bookkeeping(B, H, W, sw):
    """Every lane's 16 patch pixels come from the LDS slots that the wave's LDS-DMA filled with exactly
    that image pixel (or zeros outside the image), within the 10 KiB wave image, for every wave."""
    TH, TW = (H + 1) // 2, (W + 1) // 2
    T = B * TH * TW
    for tw0 in range(0, T, 16):
        dma, reads, total = _v2_lane_maps(tw0, T, TW, TH, H, W, sw)
        assert total <= 160
        for (r, dy, dx), pix in reads.items():
            assert 0 <= pix < 160
            t = tw0 + r
            img, rem = divmod(t, TH * TW)
            ty, tx = divmod(rem, TW)
            iy, ix = 2 * ty - 1 + dy, 2 * tx - 1 + dx
            want = (img, iy, ix) if 0 <= iy < H and 0 <= ix < W else None
            for qq in range(4):
                slot = pix * 4 + qq
                assert dma[_wino_sw(slot) if sw else slot] == want, (tw0, r, dy, dx)


def test_wino_v2_swizzle_is_a_bank_row_involution():
    for s in range(640):
        t = _wino_sw(s)
        assert t >> 4 == s >> 4 and _wino_sw(t) == s


def _sk_plan(units, kc, mult):
    """conv_wino_f32.hip conv_wino_sk_plan, transcribed."""
    total = units * kc
    G = min(256 * max(mult, 1), total)
    it = -(-total // G)
    G = -(-total // it)
    smax = max(((u + 1) * kc - 1) // it - (u * kc) // it + 1 for u in range(units))
    return G, it, smax


def _sk_segments(units, kc, G, it):
    """Every block's (unit, chunk range, partial index, partials) as the stream-K kernel walks them."""
    segs = []
    for b in range(G):
        i, end = b * it, min(units * kc, (b + 1) * it)
        while i < end:
            u, kb = divmod(i, kc)
            ke = min(kc, kb + end - i)
            zs, ns = 0, 1
            if kb or ke != kc:
                g0, g1 = (u * kc) // it, ((u + 1) * kc - 1) // it
                zs, ns = b - g0, g1 - g0 + 1
            segs.append((u, kb, ke, zs, ns))
            i += ke - kb
    return segs


@pytest.mark.parametrize("cfg_nw_fn", [(110, 8, 2), (112, 4, 1), (114, 8, 1)])
@pytest.mark.parametrize("B,H,C,N", [(32, 56, 64, 64), (32, 28, 128, 128), (32, 14, 256, 256), (32, 7, 512, 512),
                                     (2, 56, 64, 64), (3, 14, 256, 96)])
@pytest.mark.parametrize("mult", [1, 2])
def test_wino_stream_k_plan_partitions_every_unit(cfg_nw_fn, B, H, C, N, mult):
    """The stream-K walk covers each unit's K chunks exactly once, its partials are numbered 0..ns-1
    in chunk order with one agreed ns, and the ResNet-50 bs=32 shapes need <= 4 partials at 256
    blocks (the fused fixup's limit; the host refuses more)."""
    _, nw, fn = cfg_nw_fn
    if N % (16 * fn):
        pytest.skip("channels")
    T = B * ((H + 1) // 2) ** 2
    units = -(-T // (16 * nw)) * (N // (16 * fn))
    kc = C // 16
    G, it, smax = _sk_plan(units, kc, mult)
    cover = {}
    for u, kb, ke, zs, ns in _sk_segments(units, kc, G, it):
        cover.setdefault(u, []).append((kb, ke, zs, ns))
    assert sorted(cover) == list(range(units))
    for u, parts in cover.items():
        parts.sort()
        assert parts[0][0] == 0 and parts[-1][1] == kc
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        assert [p[2] for p in parts] == list(range(len(parts)))
        assert all(p[3] == len(parts) for p in parts)
        assert len(parts) <= smax
    if B == 32 and mult == 1:
        assert smax <= 4
