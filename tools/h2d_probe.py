import torch, time
n = 1 << 30
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device='cuda')
for _ in range(3): d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10): d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
el = (time.perf_counter() - t) / 10
print("1 stream H2D GB/s", n / el / 1e9)
# two streams, halves
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    with torch.cuda.stream(s1): d[: n // 2].copy_(h[: n // 2], non_blocking=True)
    with torch.cuda.stream(s2): d[n // 2:].copy_(h[n // 2:], non_blocking=True)
torch.cuda.synchronize()
el = (time.perf_counter() - t) / 10
print("2 streams H2D GB/s", n / el / 1e9)
# 64 MiB chunks on one stream
c = 64 << 20
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    for o in range(0, n, c): d[o:o + c].copy_(h[o:o + c], non_blocking=True)
torch.cuda.synchronize()
el = (time.perf_counter() - t) / 10
print("64MiB chunks H2D GB/s", n / el / 1e9)
