"""CPU checks of the producer / consumer Winograd F(4x4, 3x3) kernel's bookkeeping
(csrc/kernels/conv_wino4pc_f32.hip, cfg 210), transcribed from the kernel: the block image the producers'
LDS-DMA fills, every producer lane's patch reads, the bank behaviour of those reads and of the V-buffer
stores / consumer reads (MI355X_MICROARCH.md LDS table: ds_read_b32 / ds_write_b32 serve lanes 0-31 and
32-63 in one LDS cycle each, bank = dword mod 32), and the host's piece count."""
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C


def _geom(bx, T, TW):
    """pc_geom: the block's tile-row segments."""
    tw0 = bx * 32
    tlast = min(tw0 + 31, T - 1)
    R0 = tw0 // TW
    lo0 = tw0 - R0 * TW
    R1 = tlast // TW
    nseg = R1 - R0 + 1
    n0 = tlast - tw0 + 1 if nseg == 1 else TW - lo0
    nl = tlast - R1 * TW + 1
    pitch0, pitchm, pitchl = 9 * n0 + 4, 9 * TW + 4, 9 * nl + 4
    size0, sizem = 6 * pitch0, 6 * pitchm
    base1 = size0 + ((9 * n0 - size0) & 7)
    Sp = sizem + ((9 * TW - sizem) & 7)
    units = size0 if nseg == 1 else base1 + (nseg - 2) * Sp + 6 * pitchl
    g = dict(tw0=tw0, tlast=tlast, R0=R0, lo0=lo0, nseg=nseg, pitch0=pitch0, pitchm=pitchm, pitchl=pitchl,
             base1=base1, Sp=Sp, units=units)

    def seg(sg):
        base = 0 if sg == 0 else base1 + (sg - 1) * Sp
        pitch = pitch0 if sg == 0 else (pitchl if sg == nseg - 1 else pitchm)
        return base, pitch, (lo0 if sg == 0 else 0)
    return g, seg


def _pieces(B, H, W):
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    return -(-max(_geom(bx, T, TW)[0]["units"] for bx in range(-(-T // 32))) // 64)


def _block_maps(bx, B, H, W):
    """(dma: unit -> (img, iy, ix, half) or None, reads: (tile, ch, dy, dx) -> dword address, pieces)."""
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    g, seg = _geom(bx, T, TW)
    pieces = -(-g["units"] // 64)
    dma = {}
    for pw in range(4):
        for ii in range(11):
            i = 4 * ii + pw
            if i >= pieces:
                continue
            for lane in range(64):
                u = i * 64 + lane
                sg = 0
                if g["nseg"] > 1 and u >= g["base1"]:
                    sg = min(1 + (u - g["base1"]) // g["Sp"], g["nseg"] - 1)
                base, pitch, lo = seg(sg)
                local = u - base
                row, uu = divmod(local, pitch)
                g9, e = divmod(uu, 9)
                px, hh = 4 * g9 + (e >> 1), e & 1
                R = g["R0"] + sg
                im, ty = divmod(R, TH)
                iy, ix = 4 * ty - 1 + row, 4 * lo - 1 + px
                ok = u < g["units"] and row < 6 and e != 8 and 0 <= iy < H and 0 <= ix < W
                assert u not in dma
                dma[u] = (im, iy, ix, hh) if ok else None
    reads = {}
    for tl in range(32):
        t = g["tw0"] + tl
        if t > g["tlast"]:
            continue
        R = t // TW
        sg = R - g["R0"]
        base, pitch, lo = seg(sg)
        cgl = t - R * TW - lo
        for ch in range(8):
            rd = (base + 9 * cgl + (ch >> 2)) * 16 + (ch & 3) * 4
            for dy in range(6):
                for dx in range(6):
                    reads[(tl, ch, dy, dx)] = rd + dy * pitch * 16 + 16 * (2 * dx if dx < 4 else 2 * dx + 1)
    return dma, reads, pieces


SHAPES = [(32, 56, 56), (32, 28, 28), (32, 14, 14), (32, 7, 7), (3, 9, 13), (2, 8, 8), (5, 12, 7), (1, 4, 4)]


@pytest.mark.parametrize("B,H,W", SHAPES)
def test_wino4pc_block_image_bookkeeping(B, H, W):
    """Every producer lane's patch pixel comes from the image unit the block's LDS-DMA filled with exactly
    that input pixel and 4-channel half (zeros outside the map), within the staged pieces."""
    pieces = _pieces(B, H, W)
    assert 0 < pieces <= 43
    assert C.kernels().conv_wino4pc_pieces(B, H, W) == pieces
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    for bx in range(-(-T // 32)):
        dma, reads, pb = _block_maps(bx, B, H, W)
        assert pb <= pieces
        for (tl, ch, dy, dx), addr in reads.items():
            t = bx * 32 + tl
            im, rem = divmod(t, TH * TW)
            ty, tx = divmod(rem, TW)
            iy, ix = 4 * ty - 1 + dy, 4 * tx - 1 + dx
            want = (im, iy, ix, ch >> 2) if 0 <= iy < H and 0 <= ix < W else None
            assert addr % 16 == (ch & 3) * 4
            assert dma[addr // 16] == want, (bx, tl, ch, dy, dx)


@pytest.mark.parametrize("B,H,W,worst_ok", [(32, 56, 56, 2), (32, 28, 28, 2), (32, 14, 14, 2), (32, 7, 7, 1)])
def test_wino4pc_patch_read_banks(B, H, W, worst_ok):
    """Producer pw's lane l reads tile 16 (pw & 1) + l // 4, channel 4 (pw >> 1) + l % 4: a 32-lane group is 8
    tiles x 4 channels, 8 unit phases x 4 dwords = 32 banks inside a segment (aligned bases keep the phase
    across a boundary on the boundary's first row; other rows of a partial segment meet 2-way at worst)."""
    TH, TW = (H + 3) // 4, (W + 3) // 4
    T = B * TH * TW
    worst = 0
    for bx in range(-(-T // 32)):
        _, reads, _ = _block_maps(bx, B, H, W)
        for pw in range(4):
            for grp in range(2):
                lanes = range(32 * grp, 32 * grp + 32)
                for dy in range(6):
                    for dx in range(6):
                        banks = {}
                        for l in lanes:
                            key = (16 * (pw & 1) + l // 4, 4 * (pw >> 1) + l % 4, dy, dx)
                            if key in reads:
                                a = reads[key]
                                banks.setdefault((a // 4) % 32, set()).add(a)
                        if banks:
                            worst = max(worst, max(len(v) for v in banks.values()))
    assert worst <= worst_ok


def test_wino4pc_v_buffer_banks():
    """V[pos][s][q][t ^ 16 (q & 1)] (channel 2 q + s): the producers' ds_write_b32 meet at most 2-way (free
    for 4-byte stores), the consumers' ds_read_b32 (lane = i + 16 q, tile 16 tb + i) never."""
    def vdw(t, ch, pos=0):
        q, s = ch >> 1, ch & 1
        return (pos * 8 + s * 4 + q) * 32 + (t ^ (16 * (q & 1)))
    for pw in range(4):
        for grp in range(2):
            banks = {}
            for l in range(32 * grp, 32 * grp + 32):
                t, ch = 16 * (pw & 1) + l // 4, 4 * (pw >> 1) + l % 4
                a = vdw(t, ch)
                banks.setdefault(a % 32, set()).add(a)
            assert max(len(v) for v in banks.values()) <= 2
    for tb in range(2):
        for s in range(2):
            for grp in range(2):
                banks = {}
                for l in range(32 * grp, 32 * grp + 32):
                    i, q = l & 15, l >> 4
                    a = (s * 4 + q) * 32 + ((tb ^ (q & 1)) * 16 + i)
                    assert a == vdw(16 * tb + i, 2 * q + s)
                    banks.setdefault(a % 32, set()).add(a)
                assert max(len(v) for v in banks.values()) == 1


def test_wino4pc_registered():
    assert 210 in C.WINO4_F32_CFGS
    assert C.wino4_map_ok(32, 7, 7, 210) and C.wino4_map_ok(1, 4, 4, 210)
