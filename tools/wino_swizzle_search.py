#!/usr/bin/env python3
"""Bank-conflict model of conv_wino_f32_v2's patch reads (csrc/kernels/conv_wino_f32.hip).

Each wave stages <= 160 input pixels (16 channels = four 16-B quads each) in its
own LDS image by LDS-DMA; lane (r, q) then reads quad q of the 16 patch pixels of
tile r with ds_read_b128.  Unswizzled, pixel P quad q sits in 16-B slot 4P + q,
so the slot's position in its 256-B bank row is 4(P & 3) + q: consecutive tiles
are 2 pixels apart and a 16-lane ds_read_b128 group hits only 4 positions (4-way).
The swizzle XORs the position with h(row), row = slot >> 4 (a bijection inside
each bank row, so the DMA side just inverts it per lane).  This script walks every
wave of the four ResNet-50 shapes and reports the LDS cycles per chunk per wave
for candidate h, using the ds_read_b128 lane groups of MI355X_MICROARCH.md §LDS.
"""
import itertools

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def wave_patch_pixels(T, TW, TH, B, tw0):
    """Per lane r (tile tw0 + r): the image pixel index of patch (dy, dx), as the kernel lays segments out."""
    tlast = min(tw0 + 15, T - 1)
    R0 = tw0 // TW
    nseg = tlast // TW - R0 + 1
    seg_lo, seg_w, seg_b = [], [], [0]
    for sg in range(4):
        lo = tw0 - R0 * TW if sg == 0 else 0
        hi = tlast - (R0 + sg) * TW if sg == nseg - 1 else TW - 1
        seg_lo.append(lo)
        seg_w.append(2 * (hi - lo + 1) + 2 if sg < nseg else 0)
        seg_b.append(seg_b[-1] + 4 * seg_w[-1])
    assert seg_b[nseg] <= 160, (TW, tw0, seg_b)
    out = []
    for r in range(16):
        t = tw0 + r
        if t >= T:
            out.append(None)
            continue
        tsg = t // TW - R0
        pw, pb0, plo = seg_w[tsg], seg_b[tsg], seg_lo[tsg] if tsg == 0 else 0
        prow0 = pb0 + 2 * (t - (R0 + tsg) * TW - plo)
        out.append([prow0 + dy * pw + dx for dy in range(4) for dx in range(4)])
    return out


def pos(P, q, h):
    s = 4 * P + q
    row = s >> 4
    return row, (s & 15) ^ h(row)


def cycles_for_wave(pix, h):
    total = 0
    for k in range(16):
        for g in GROUPS:
            slots = {}
            for l in g:
                r, q = l & 15, l >> 4
                if pix[r] is None:
                    continue
                row, w = pos(pix[r][k], q, h)
                slots.setdefault(w, set()).add(row)
            total += max((len(v) for v in slots.values()), default=1)
    return total


SHAPES = {"stage2": (56, 32), "stage3": (28, 32), "stage4": (14, 32), "stage5": (7, 32)}


def evaluate(h, waves_per_shape=None):
    res = {}
    for name, (Hs, B) in SHAPES.items():
        TH = TW = (Hs + 1) // 2
        T = B * TH * TW
        nw = (T + 15) // 16
        idx = range(nw) if waves_per_shape is None else range(0, nw, max(1, nw // waves_per_shape))
        c = [cycles_for_wave(wave_patch_pixels(T, TW, TH, B, w * 16), h) for w in idx]
        res[name] = sum(c) / len(c)
    return res


if __name__ == "__main__":
    base = evaluate(lambda row: 0, 200)
    print("unswizzled  ", {k: round(v, 1) for k, v in base.items()}, "(ideal 64)")
    cands = {}
    for a, b, sh in itertools.product(range(16), range(16), range(0, 4)):
        h = (lambda a, b, sh: (lambda row: (a * row + b * (row >> sh)) & 15))(a, b, sh)
        cands[(a, b, sh)] = h
    scored = []
    for key, h in cands.items():
        r = evaluate(h, 60)
        scored.append((sum(r.values()), key, r))
    scored.sort()
    for s, key, r in scored[:8]:
        print("h(row) = (%d*row + %d*(row>>%d)) & 15" % key, {k: round(v, 1) for k, v in r.items()})
    best = scored[0][1]
    print("full check of the best:", {k: round(v, 1) for k, v in evaluate(cands[best]).items()})
