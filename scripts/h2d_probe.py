"""H2D probe: pinned host -> device copy rate at the config-5 frame size, alone and
with the decode, to see what bounds bench.py's stream_h2d (diagnostic)."""
import time
import torch

dev = torch.device("cuda", 0)
n = 2_120_000
for nbytes, reps in ((n, 256), (8 * n, 64), (64 * n, 8)):
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        for _ in range(4):
            d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        e0.record(s)
        for _ in range(reps):
            d.copy_(h, non_blocking=True)
        e1.record(s)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    print(f"{nbytes/1e6:8.2f} MB x{reps}: gpu {nbytes*reps/e0.elapsed_time(e1)/1e6:7.2f} GB/s, "
          f"wall {nbytes*reps/wall/1e9:7.2f} GB/s, issue {t_issue/reps*1e6:7.1f} us/copy")
