import torch, time
x = torch.zeros(1, device="cuda")
big = torch.zeros(196*256, device="cuda")
def t(fn, n=20):
    fn(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n): fn()
    g.replay(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10): g.replay()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / (10 * n) * 1000
print("1-element add_ per launch (us):", round(t(lambda: x.add_(1)), 2))
print("50k-element add_ (196 WGs) per launch (us):", round(t(lambda: big.add_(1)), 2))
