import itertools
W, TR = 28, 4
HW2 = W + 2
PX = TR * W
PF = (PX + 15) // 16
groups = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32)),
          [l+32 for l in list(range(0,4))+list(range(12,16))+list(range(20,28))], [l+32 for l in list(range(4,12))+list(range(16,20))+list(range(28,32))]]
def cost(slot):
    tot = 0
    for f in range(PF):
        for tap in range(9):
            toff = (tap // 3) * HW2 + tap % 3
            for cc in range(4):
                for g in groups:
                    seen = {}
                    for l in g:
                        fr, fq = l & 15, l >> 4
                        px = min(f * 16 + fr, PX - 1)
                        r = (px // W) * HW2 + px % W + toff
                        c = cc * 4 + fq
                        s = slot(r, c)
                        seen.setdefault(s, set()).add((r, c))
                    tot += max(len(v) for v in seen.values()) - 1
    return tot
cands = {
 "xor r&15": lambda r, c: c ^ (r & 15),
 "pad272 (r+c)": lambda r, c: (r + c) & 15,
 "xor 3r": lambda r, c: c ^ ((3 * r) & 15),
 "xor 5r": lambda r, c: c ^ ((5 * r) & 15),
 "xor 7r": lambda r, c: c ^ ((7 * r) & 15),
 "xor 9r": lambda r, c: c ^ ((9 * r) & 15),
 "add 3r": lambda r, c: (c + 3 * r) & 15,
 "add 5r": lambda r, c: (c + 5 * r) & 15,
 "add 7r": lambda r, c: (c + 7 * r) & 15,
 "add 9r": lambda r, c: (c + 9 * r) & 15,
 "add 4r": lambda r, c: (c + 4 * r) & 15,
 "add 2r": lambda r, c: (c + 2 * r) & 15,
 "xor (r<<1 | r>>3)": lambda r, c: c ^ (((r << 1) | ((r >> 3) & 1)) & 15),
}
for k, fn in cands.items():
    print(f"{k:22s} extra cycles {cost(fn)}")
print("---- search")
best = []
for a in range(16):
    for b in (1, 3, 5, 7, 9, 11, 13, 15):
        best.append((cost(lambda r, c, a=a, b=b: (a * r + b * c) & 15), f"add a={a} b={b}"))
        best.append((cost(lambda r, c, a=a, b=b: ((b * c) & 15) ^ ((a * r) & 15)), f"xor a={a} b={b}"))
for sh in range(1, 5):
    for a in range(16):
        best.append((cost(lambda r, c, a=a, sh=sh: c ^ ((a * r + (r >> sh)) & 15)), f"xor a*r+(r>>{sh}) a={a}"))
        best.append((cost(lambda r, c, a=a, sh=sh: (c + a * r + (r >> sh)) & 15), f"add a*r+(r>>{sh}) a={a}"))
best.sort()
print(best[:8])
