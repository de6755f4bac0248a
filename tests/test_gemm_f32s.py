"""CPU checks of the fp32 big-tile 1x1 GEMM's bookkeeping (csrc/kernels/gemm_f32s.hip, cfg ids 300+): the LDS
swizzle of a K chunk (the LDS-DMA lane that fills a slot fetches the unit the fragment read expects there), the
bank behaviour of the fragment reads (MI355X_MICROARCH.md LDS table: ds_read_b128 serves 4 groups of 16 lanes,
{0-3,12-15,20-27}, {4-11,16-19,28-31}, +32; a group is conflict-free when its 16 lanes hit 16 distinct 16-byte
slots of the 256-byte bank row), the stream-K ranges and slots, and the host tables."""
import pytest

from adaptive_deep_learning_architecture_for_parallel_and_fault_tolerant_inference_amd.ops import conv as C


def swz(r, c):
    return r * 128 + ((c ^ ((r >> 1) & 7)) << 4)


def test_dma_fills_what_the_reads_expect():
    """DMA lane l of piece pi writes LDS byte pi*1024 + 16 l = row 8 pi + l // 8, slot l % 8, fetching logical unit
    (l % 8) ^ ((row >> 1) & 7); the read of (row, unit) at swz(row, unit) finds exactly that unit."""
    filled = {}
    for pi in range(60):
        for lane in range(64):
            r = pi * 8 + (lane >> 3)
            c = (lane & 7) ^ ((r >> 1) & 7)
            filled[pi * 1024 + 16 * lane] = (r, c)
    for r in range(480):
        for c in range(8):
            assert filled[swz(r, c)] == (r, c)


GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


@pytest.mark.parametrize("row0", [0, 16, 112, 240, 464])
@pytest.mark.parametrize("h", [0, 1])
def test_fragment_reads_conflict_free(row0, h):
    for g in GROUPS:
        slots = set()
        for lane in g:
            i, q = lane & 15, lane >> 4
            slots.add((swz(row0 + i, 4 * h + q) // 16) % 16)
        assert len(slots) == 16, (row0, h, g)


def _ranges(U, G):
    return [(v * U // G, (v + 1) * U // G) for v in range(G)]


@pytest.mark.parametrize("tiles,KT", [(56, 8), (49, 32), (26, 64), (224, 4), (14, 64)])
def test_stream_k_slots(tiles, KT):
    """Every (tile, chunk) unit is run once; the kernel's contributor range and slot rule of a split tile name
    exactly the blocks that wrote partials of it, each slot written once."""
    G = 256
    U = tiles * KT
    per = U // G
    if per < 1 or -(-KT // per) + 1 > 16:
        pytest.skip("the host rejects it: fewer units than blocks, or > 16 blocks on one tile")
    rng = _ranges(U, G)
    seen = [0] * U
    written = {}
    for v, (u0, u1) in enumerate(rng):
        u = u0
        while u < u1:
            t, c0 = divmod(u, KT)
            c1 = min(KT, c0 + (u1 - u))
            for k in range(t * KT + c0, t * KT + c1):
                seen[k] += 1
            if not (c0 == 0 and c1 == KT):
                slot = 2 * v + (0 if u == u0 else 1)
                assert slot not in written
                written[slot] = t
            u += c1 - c0
    assert seen == [1] * U
    vof = lambda u: ((u + 1) * G - 1) // U
    for t in range(tiles):
        vf, vl = vof(t * KT), vof(t * KT + KT - 1)
        if vf == vl and rng[vf][0] <= t * KT and rng[vf][1] >= (t + 1) * KT:
            assert t not in written.values()
            continue
        slots = [2 * w + (0 if rng[w][0] >= t * KT else 1) for w in range(vf, vl + 1)]
        assert sorted(slots) == sorted(s for s, tt in written.items() if tt == t)
        assert vl - vf + 1 <= 16


def test_tables():
    for cfg, (bm, bn) in C.F32S_CFGS.items():
        assert tuple(C.kernels().gemm_f32s_cfg(cfg)) == (bm, bn)
        assert C.kernels().gemm_f32s_ws_elems(cfg) == C.f32s_ws_elems(cfg)
    assert C.f32s_tiles(300, 6272, 256) == 56 and C.f32s_tiles(300, 25088, 512) == 448
