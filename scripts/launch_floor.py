"""Back-to-back launch floor on this GPU (diagnostic): a hipGraph of K tiny torch
kernels replayed, per-kernel time = region / K. The single-frame decode cannot
go below this."""
import torch

K = 200
x = torch.zeros(1, device="cuda")
big = torch.zeros(768 * 512, device="cuda")
for name, fn in [("tiny add (1 WG)", lambda: x.add_(1)),
                 ("fill 768x512 thr", lambda: big.add_(1))]:
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(K):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) * 1e3 / (10 * K):.3f} us per kernel")
