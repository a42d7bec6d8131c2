"""PCIe copy rates on the box (tool, not product): pinned host <-> device, the sizes the C2/C4
pipelines move per batch (16 MB of 16-byte query records, 1 MB decisions, 4 MB errors)."""
import time

import torch

dev = torch.device("cuda:0")
for mb in (1, 4, 16, 32, 64):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    for direction in ("h2d", "d2h"):
        for _ in range(3):
            (d.copy_(h, non_blocking=True) if direction == "h2d" else h.copy_(d, non_blocking=True))
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            (d.copy_(h, non_blocking=True) if direction == "h2d" else h.copy_(d, non_blocking=True))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(f"{direction} {mb:3d} MB: {dt * 1e3:7.3f} ms  {n / dt / 1e9:6.1f} GB/s", flush=True)
# both directions at once on two streams
n = 16 << 20
h1, h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True), torch.empty(n, dtype=torch.uint8, pin_memory=True)
d1, d2 = torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    with torch.cuda.stream(s1):
        d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
print(f"h2d+d2h 16 MB each, two streams: {dt * 1e3:.3f} ms ({2 * n / dt / 1e9:.1f} GB/s total)", flush=True)
